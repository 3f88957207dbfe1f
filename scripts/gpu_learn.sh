#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/learning_curve.py --steps ${STEPS:-30000} --envs 65536 --every ${EVERY:-1000} -o gpurun_out/learning.md > gpurun_out/learning.log 2>&1
rc=$?; cat gpurun_out/learning.md; exit $rc
