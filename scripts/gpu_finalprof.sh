#!/bin/bash
# Current-state profiles: PMC passes, phase stamps, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 bash scripts/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_run.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/stamp_qstep.py --out gpurun_out/stamps_final.md > gpurun_out/stamps_final.log 2>&1
rc=$?; cat gpurun_out/stamps_final.md; exit $rc
