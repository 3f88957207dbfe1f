#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gru
for g in ${GRIDS:-256 224 192 160}; do
  for m in ${MODES:-"" "--no-overlap-act"}; do
    tag=$(echo "g$g$m" | tr -d ' -')
    timeout -k 10 200 python benchmarks/bench_gru.py --grid $g $m > gpurun_out/gru/$tag.log 2>&1 || exit $?
    echo "[grid $g $m] $(tail -1 gpurun_out/gru/$tag.log | grep -oE '"ms_per_iteration": [0-9.]+|"act_ms": [0-9.]+|"update_ms": [0-9.]+' | tr '\n' ' ')"
  done
done
