#!/bin/bash
# 1-GPU bench at several envs-per-GPU counts (per-GPU work per step vs fixed per-step overheads).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/envsweep
for e in ${ENVS:-32768 65536 131072 262144}; do
  timeout -k 10 240 python bench.py --envs $e --steps 500 --warmup 50 > gpurun_out/envsweep/e$e.log 2>&1 || exit $?
  tail -1 gpurun_out/envsweep/e$e.log | cut -c1-260
done
