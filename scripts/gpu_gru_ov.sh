#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gru
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gru/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/gru/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in "" "--no-overlap-act"; do
    tag=$(echo "x$m" | tr -d ' -')
    timeout -k 10 200 python benchmarks/bench_gru.py $m > gpurun_out/gru/$tag.$rep.log 2>&1 || exit $?
    echo "[$m] rep$rep $(tail -1 gpurun_out/gru/$tag.$rep.log | grep -oE '"ms_per_iteration": [0-9.]+|"env_steps_per_s": [0-9.]+|"updates_per_s": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+|"loss": [0-9.e-]+' | tr '\n' ' ')"
  done
done
