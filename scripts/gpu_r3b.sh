#!/bin/bash
# round 3: the new wave-specialised step kernel first (own process, short limit), then the GPU suite,
# then the default bench and the bench on the new kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_qstep_ws.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r3b_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3b_ws.log; exit 1; }
tail -5 gpurun_out/r3b_ws.log
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --step-kernel ws --no-episode > gpurun_out/r3b_bench_ws.log 2>&1 \
  || { echo BENCHWS_FAIL; tail -30 gpurun_out/r3b_bench_ws.log; exit 1; }
tail -1 gpurun_out/r3b_bench_ws.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rs \
  --ignore=tests/test_gpu_qstep_ws.py > gpurun_out/r3b_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r3b_pytest.log; exit 1; }
tail -4 gpurun_out/r3b_pytest.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3b_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r3b_bench.log; exit 1; }
tail -1 gpurun_out/r3b_bench.log
