#!/bin/bash
# round 3: batch-1 learner host path (double-buffered staging, cached launch structs) -- tests, latency, reference app
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_app.py tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 \
  || { echo TEST_FAIL; tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -1 gpurun_out/r4p_tests.log
timeout -k 10 200 python -u tools/learner_latency.py > gpurun_out/r4p_latency.log 2>&1 || { echo LAT_FAIL; tail -20 gpurun_out/r4p_latency.log; exit 1; }
tail -1 gpurun_out/r4p_latency.log
timeout -k 10 300 python -u benchmarks/bench_app.py --engine actors > gpurun_out/r4p_app.log 2>&1 || { echo APP_FAIL; tail -20 gpurun_out/r4p_app.log; exit 1; }
grep '^{' gpurun_out/r4p_app.log | cut -c1-500
