#!/bin/bash
# How the timed window's length and warmup affect bench.py (driver runs --steps 20 --warmup 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "20 5" "20 50" "20 200" "100 5" "300 30" "20 5"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 > gpurun_out/short_$1_$2.log 2>&1 || exit $?
  echo "steps=$1 warmup=$2 $(tail -1 gpurun_out/short_$1_$2.log | grep -oE '"ms_per_step": [0-9.]+')"
done
