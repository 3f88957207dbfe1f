#!/bin/bash
# round 3: ws kernel v2 -- numerics first, then stamps + bench, then the whole GPU suite (no -x)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_qstep_ws.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3c_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3c_ws.log; exit 1; }
tail -3 gpurun_out/r3c_ws.log
timeout -k 10 120 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r3c_stamps_ws.md \
  > gpurun_out/r3c_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3c_stamps.log; exit 1; }
cat gpurun_out/r3c_stamps_ws.md
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --step-kernel ws --no-episode > gpurun_out/r3c_bench_ws.log 2>&1 \
  || { echo BENCHWS_FAIL; tail -30 gpurun_out/r3c_bench_ws.log; exit 1; }
tail -1 gpurun_out/r3c_bench_ws.log | cut -c1-400
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rs \
  --ignore=tests/test_gpu_qstep_ws.py > gpurun_out/r3c_pytest.log 2>&1; echo "pytest rc=$?"
tail -15 gpurun_out/r3c_pytest.log
