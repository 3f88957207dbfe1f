#!/bin/bash
# round 3: GPU test suite + default bench (with the full-episode returns)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rs \
  > gpurun_out/r3a_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r3a_pytest.log; exit 1; }
tail -4 gpurun_out/r3a_pytest.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3a_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r3a_bench.log; exit 1; }
tail -2 gpurun_out/r3a_bench.log
