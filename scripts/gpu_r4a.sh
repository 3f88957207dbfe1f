#!/bin/bash
# round 3 checkpoint: full GPU suite, default bench, smoke, stamps of the production ws kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 > gpurun_out/r4a_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r4a_bench.log; exit 1; }
tail -1 gpurun_out/r4a_bench.log | cut -c1-900
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4a_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r4a_suite.log; exit 1; }
tail -2 gpurun_out/r4a_suite.log
timeout -k 10 60 python -u __graft_entry__.py smoke > gpurun_out/r4a_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r4a_smoke.log; exit 1; }
tail -1 gpurun_out/r4a_smoke.log | cut -c1-200
timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r4a_stamps_ws.md \
  > gpurun_out/r4a_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r4a_stamps.log; exit 1; }
cat gpurun_out/r4a_stamps_ws.md
