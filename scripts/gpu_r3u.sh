#!/bin/bash
# round 3: wave issue priority (data waves over gradient waves and the reverse)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in "" dprio gprio; do
  extra="--step-kernel ws"; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode $extra > gpurun_out/r3u_bench_${v}_$rep.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r3u_bench_${v}_$rep.log; exit 1; }
  echo "$v $rep: $(tail -1 gpurun_out/r3u_bench_${v}_$rep.log | cut -c100-200)"
done
done
