#!/bin/bash
# Serving path: kernel numerics tests, serving benchmark, kernel trace of the benchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/serve
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_serve.py -x -v --timeout 120 --timeout-method thread > gpurun_out/serve/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/serve/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_serve.py > gpurun_out/serve/bench.log 2>&1
rc=$?; cat gpurun_out/serve/bench.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/serve/prof" -o run -- python3 "$R/benchmarks/bench_serve.py" --batches 1024,131072 --clients 8 --requests 20 > "$R/gpurun_out/serve/prof.log" 2>&1
rc=$?; tail -1 "$R/gpurun_out/serve/prof.log" | cut -c1-150; exit $rc
