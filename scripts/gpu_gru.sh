#!/bin/bash
# Config 5 call: GRU tests, benchmark and a rocprofv3 kernel-trace of the benchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python benchmarks/bench_gru.py ${GRU_ARGS:-} > gpurun_out/bench_gru.log 2>&1
rc=$?; tail -2 gpurun_out/bench_gru.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profgru" -o run -- python3 "$R/benchmarks/bench_gru.py" --steps 5 --warmup 2 ${GRU_ARGS:-} > "$R/gpurun_out/profgru.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/profgru.log"; exit $rc
