#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/rtrace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/rtrace" -o run -- python3 "$R/tools/overlap_rehearsal.py" --steps 30 --warmup 5 --usec 25 --cus 8 > "$R/gpurun_out/rtrace.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/rtrace.log"; find "$R/gpurun_out/rtrace" -name "*.csv" | head; exit $rc
