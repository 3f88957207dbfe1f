#!/bin/bash
# config 4: tests + A/B of overlapped act step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/deep
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/deep/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/deep/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in "" "--overlap-act"; do
    tag=$(echo "x$m" | tr -d ' -')
    timeout -k 10 200 python benchmarks/bench_deep.py $m > gpurun_out/deep/ov_$tag.$rep.log 2>&1 || exit $?
    echo "[$m] rep$rep $(tail -1 gpurun_out/deep/ov_$tag.$rep.log | grep -oE '"ms_per_iteration": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+|"mean_loss": [0-9.e-]+' | tr '\n' ' ')"
  done
done
