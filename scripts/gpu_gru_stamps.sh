#!/bin/bash
# Phase stamps of the single- and two-chunk GRU actor kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/grupair
for k in single pair; do
  timeout -k 10 200 python tools/stamp_gru.py --kernel $k --out gpurun_out/grupair/stamps_$k.md > gpurun_out/grupair/stamps_$k.log 2>&1 || exit $?
  cat gpurun_out/grupair/stamps_$k.md
done
