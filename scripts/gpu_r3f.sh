#!/bin/bash
# round 3: ws kernel (packed relu, pipelined layer loops) -- numerics + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_qstep_ws.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3f_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3f_ws.log; exit 1; }
tail -2 gpurun_out/r3f_ws.log
for i in 1 2; do
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-episode > gpurun_out/r3f_bench_ws_$i.log 2>&1 \
  || { echo BENCHWS_FAIL; tail -30 gpurun_out/r3f_bench_ws_$i.log; exit 1; }
tail -1 gpurun_out/r3f_bench_ws_$i.log | cut -c1-240
done
