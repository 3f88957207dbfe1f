#!/bin/bash
# Configs 4 and 5 benchmarks on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bench_deep.py > gpurun_out/bench_deep.log 2>&1
rc=$?; tail -1 gpurun_out/bench_deep.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_gru.py > gpurun_out/bench_gru.log 2>&1
rc=$?; tail -1 gpurun_out/bench_gru.log | cut -c1-900; exit $rc
