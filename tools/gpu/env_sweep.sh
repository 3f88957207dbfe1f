#!/bin/bash
# flagship env-count sweep at the driver's step counts (ws kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5sweep}
mkdir -p $D
for E in 1835008 2752512 3670016 1835008; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-episode --envs $E > $D/bench_$E.log 2>&1 || exit 1
  echo "$E $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$E.log) $(grep -o '"value": [0-9.]*' $D/bench_$E.log) $(grep -o '"hbm_used_gb": [0-9.]*' $D/bench_$E.log)"
done
