#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
rm -rf gpurun_out/gruprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/gruprof" -o run -- python3 "$R/benchmarks/bench_gru.py" --steps 5 > "$R/gpurun_out/gruprof.log" 2>&1
rc=$?; tail -1 "$R/gpurun_out/gruprof.log" | cut -c1-200; exit $rc
