#!/bin/bash
# GEMM + config-4 tests, then config-4 bench (new tile choice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/deep
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_deep.py tests/test_gpu_gru.py -x -q --timeout 120 --timeout-method thread > gpurun_out/deep/pytest_tile.log 2>&1
rc=$?; tail -2 gpurun_out/deep/pytest_tile.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python benchmarks/bench_deep.py > gpurun_out/deep/tile.$rep.log 2>&1 || exit $?
  echo "rep$rep $(tail -1 gpurun_out/deep/tile.$rep.log | grep -oE '"ms_per_iteration": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+' | tr '\n' ' ')"
done
timeout -k 10 200 python benchmarks/bench_gru.py > gpurun_out/deep/gru.log 2>&1 || exit $?
tail -1 gpurun_out/deep/gru.log | grep -oE '"[a-z_]*ms[a-z_]*": [0-9.]+|"env_steps_per_s": [0-9.]+|"updates_per_s": [0-9.]+' | tr '\n' ' '
