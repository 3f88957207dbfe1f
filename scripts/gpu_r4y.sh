#!/bin/bash
# round 3: layer-1 W0 read-ahead 8 / 10 / 12 pairs on the final kernel -- numerics, A/B
set -o pipefail
mkdir -p gpurun_out
for v in "" pd1a pd1b; do
  SHARETRADE_WS_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4y_ws_$v.log 2>&1 || { echo WS_FAIL $v; tail -40 gpurun_out/r4y_ws_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r4y_ws_$v.log)"
done
for rep in 1 2; do
for v in "" pd1a pd1b; do
  extra="--step-kernel ws"; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode $extra > gpurun_out/r4y_bench_${v}_$rep.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r4y_bench_${v}_$rep.log; exit 1; }
  echo "$v $rep: $(tail -1 gpurun_out/r4y_bench_${v}_$rep.log | cut -c100-200)"
done
done
