#!/bin/bash
# round 3: reference app (actors engine), thread-per-neuron vs legacy fp32 GEMV, interleaved on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/r4q_tests.log; exit 1; }
tail -1 gpurun_out/r4q_tests.log
for r in 1 2; do
for g in new legacy; do
  SHARETRADE_F32_GEMV=$g timeout -k 10 200 python -u tools/learner_latency.py > gpurun_out/r4q_lat_${g}_$r.log 2>&1 || { echo LAT_FAIL; exit 1; }
  SHARETRADE_F32_GEMV=$g timeout -k 10 300 python -u benchmarks/bench_app.py --engine actors > gpurun_out/r4q_app_${g}_$r.log 2>&1 || { echo APP_FAIL; tail -20 gpurun_out/r4q_app_${g}_$r.log; exit 1; }
  echo "$g $r: $(tail -1 gpurun_out/r4q_lat_${g}_$r.log) app $(grep '^{' gpurun_out/r4q_app_${g}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["elapsed_s"])')"
done
done
