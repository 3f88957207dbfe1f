#!/bin/bash
# round 5: pipe kernel per-phase stamps at the bench geometry
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 SHARETRADE_AB_BUILDS=1
mkdir -p gpurun_out/r5c
timeout -k 10 300 python -u tools/stamp_pipe.py --out gpurun_out/r5c/stamps_pipe.md > gpurun_out/r5c/stamps.log 2>&1
rc=$?
cat gpurun_out/r5c/stamps_pipe.md
exit $rc
