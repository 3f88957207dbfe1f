#!/bin/bash
# the loader-staged ping-pong GEMM (tile "ppl") vs the production ping-pong and hipBLASLt; then config 4 with it
set -o pipefail
export PYTHONUNBUFFERED=1
D=gpurun_out/r6o
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm.py > $D/pytest_gemm.log 2>&1 || { tail -30 $D/pytest_gemm.log; exit 1; }
tail -1 $D/pytest_gemm.log
timeout -k 10 300 python tools/bench_gemm_pp.py > $D/gemm_pp.md 2>&1 || { tail -20 $D/gemm_pp.md; exit 1; }
cat $D/gemm_pp.md
