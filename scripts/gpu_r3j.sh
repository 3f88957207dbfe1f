#!/bin/bash
# round 3: ws kernel -- conflict-free H1/H2 swizzle; price the phases with timing builds (l1x2, l2x2, gskip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3j_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3j_ws.log; exit 1; }
tail -2 gpurun_out/r3j_ws.log
for v in "" gskip l1x2 l2x2; do
  extra=""; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 40 --warmup 10 --no-episode $extra > gpurun_out/r3j_bench_$v.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r3j_bench_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r3j_bench_$v.log | cut -c100-200)"
done
timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-episode > gpurun_out/r3j_bench_long.log 2>&1 \
  || { echo BENCH_FAIL long; tail -30 gpurun_out/r3j_bench_long.log; exit 1; }
echo "long: $(tail -1 gpurun_out/r3j_bench_long.log | cut -c100-200)"
