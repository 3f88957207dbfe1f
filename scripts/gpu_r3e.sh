#!/bin/bash
# round 3: ws kernel -- numerics + bench (production build, no stamp code)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_qstep_ws.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3e_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3e_ws.log; exit 1; }
tail -2 gpurun_out/r3e_ws.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --step-kernel ws --no-episode > gpurun_out/r3e_bench_ws.log 2>&1 \
  || { echo BENCHWS_FAIL; tail -30 gpurun_out/r3e_bench_ws.log; exit 1; }
tail -1 gpurun_out/r3e_bench_ws.log | cut -c1-300
timeout -k 10 120 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r3e_stamps_ws.md \
  > gpurun_out/r3e_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3e_stamps.log; exit 1; }
cat gpurun_out/r3e_stamps_ws.md
