#!/bin/bash
# round 3: refresh the secondary benchmarks on the round-3 tree (config 5, the reference app, serving)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/bench_gru.py > gpurun_out/r4n_gru.log 2>&1 || { echo GRU_FAIL; tail -20 gpurun_out/r4n_gru.log; exit 1; }
tail -1 gpurun_out/r4n_gru.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_app.py --engine both > gpurun_out/r4n_app.log 2>&1 || { echo APP_FAIL; tail -20 gpurun_out/r4n_app.log; exit 1; }
grep '^{' gpurun_out/r4n_app.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_serve.py > gpurun_out/r4n_serve.log 2>&1 || { echo SERVE_FAIL; tail -20 gpurun_out/r4n_serve.log; exit 1; }
tail -3 gpurun_out/r4n_serve.log | cut -c1-400
