#!/bin/bash
# config 4: bench + kernel trace with per-dispatch timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 200 python benchmarks/bench_deep.py > gpurun_out/deep_bench.log 2>&1
rc=$?; tail -1 gpurun_out/deep_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/deepprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/deepprof" -o run -- python3 "$R/benchmarks/bench_deep.py" --steps 10 --warmup 8 > "$R/gpurun_out/deepprof.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/deepprof.log" | cut -c1-200; exit $rc
