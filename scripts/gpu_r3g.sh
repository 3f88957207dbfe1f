#!/bin/bash
# round 3: how fast do the ws data waves run alone (gskip timing build)?  then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-episode > gpurun_out/r3g_bench_ws.log 2>&1 \
  || { echo BENCHWS_FAIL; tail -30 gpurun_out/r3g_bench_ws.log; exit 1; }
tail -1 gpurun_out/r3g_bench_ws.log | cut -c1-200
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-episode --step-kernel ws --step-variant gskip \
  > gpurun_out/r3g_bench_gskip.log 2>&1 || { echo BENCHGS_FAIL; tail -30 gpurun_out/r3g_bench_gskip.log; exit 1; }
tail -1 gpurun_out/r3g_bench_gskip.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3g_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r3g_suite.log; exit 1; }
tail -3 gpurun_out/r3g_suite.log
