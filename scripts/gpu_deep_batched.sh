#!/bin/bash
# config 4: GEMM + deep tests, then A/B of the batched forward (VARIANTS: '|'-separated bench_deep args).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/deepb
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_deep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/deepb/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/deepb/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-"|--unbatched-fwd"}
IFS='|' read -ra VS <<< "$VARIANTS"
for rep in 1 2; do
  for m in "${VS[@]}"; do
    tag=$(echo "x$m" | tr -d ' -=')
    timeout -k 10 200 python benchmarks/bench_deep.py $m > gpurun_out/deepb/$tag.$rep.log 2>&1 || exit $?
    echo "[$m] rep$rep $(tail -1 gpurun_out/deepb/$tag.$rep.log | grep -oE '"ms_per_iteration": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+' | tr '\n' ' ')"
  done
done
