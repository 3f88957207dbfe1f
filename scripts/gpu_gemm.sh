#!/bin/bash
# GEMM tests + throughput table (all tile builds vs torch.matmul).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm.py gpurun_out/gemm_tiles.md > gpurun_out/gemm_tiles.log 2>&1
rc=$?; cat gpurun_out/gemm_tiles.md; exit $rc
