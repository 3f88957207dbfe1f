#!/bin/bash
# Two-chunk GRU actor: numerics tests, then bench_gru A/B (single vs pair actor kernel, overlapped
# and serial iteration).  VARIANTS overrides the list of bench_gru argument sets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/grupair
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py -x -v --timeout 120 --timeout-method thread > gpurun_out/grupair/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/grupair/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=${VARIANTS:-"--actor-kernel=single|--actor-kernel=pair|--actor-kernel=single --no-overlap-act|--actor-kernel=pair --no-overlap-act"}
IFS='|' read -ra VS <<< "$VARIANTS"
for rep in 1 2; do
  for m in "${VS[@]}"; do
    tag=$(echo "x$m" | tr -d ' -=')
    timeout -k 10 200 python benchmarks/bench_gru.py $m > gpurun_out/grupair/$tag.$rep.log 2>&1 || exit $?
    echo "[$m] rep$rep $(tail -1 gpurun_out/grupair/$tag.$rep.log | grep -oE '"ms_per_iteration": [0-9.]+|"env_steps_per_s": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+|"actor_grid": [0-9]+' | tr '\n' ' ')"
  done
done
