#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/overlap_rehearsal.py --steps 100 --usec ${USEC:-25} --cus 0,8,32,64 -o gpurun_out/overlap.md > gpurun_out/overlap.log 2>&1
rc=$?; cat gpurun_out/overlap.md; exit $rc
