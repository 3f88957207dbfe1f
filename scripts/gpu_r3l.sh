#!/bin/bash
# round 3: ws kernel -- env-state write-back deferred past the next tile's window wait
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3l_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3l_ws.log; exit 1; }
tail -1 gpurun_out/r3l_ws.log
for v in "" pfe; do
  extra=""; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 100 --warmup 10 --no-episode $extra > gpurun_out/r3l_bench_$v.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r3l_bench_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r3l_bench_$v.log | cut -c100-200)"
done
