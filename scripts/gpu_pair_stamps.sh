#!/bin/bash
# Interval stamps of the two-slot kernel and phase stamps of the wide kernel at 1M envs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_qstep.py --envs 1048576 --kernel pair --out gpurun_out/stamps_pair.md > gpurun_out/stamps_pair.log 2>&1
rc=$?; tail -18 gpurun_out/stamps_pair.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamp_qstep.py --envs 1048576 --out gpurun_out/stamps_wide.md > gpurun_out/stamps_wide.log 2>&1
rc=$?; tail -14 gpurun_out/stamps_wide.log; exit $rc
