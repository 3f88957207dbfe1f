#!/bin/bash
# round 3 final checkpoint: full GPU suite, smoke, bench at the driver's args
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4s_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r4s_suite.log; exit 1; }
tail -1 gpurun_out/r4s_suite.log
timeout -k 10 60 python -u __graft_entry__.py smoke > gpurun_out/r4s_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r4s_smoke.log; exit 1; }
tail -1 gpurun_out/r4s_smoke.log | cut -c1-120
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4s_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r4s_bench.log; exit 1; }
tail -1 gpurun_out/r4s_bench.log | cut -c1-330
