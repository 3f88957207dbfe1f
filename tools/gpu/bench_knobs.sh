#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5kb}
mkdir -p $D
K="--target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global"
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode $K > $D/bench_knobs_$i.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $D/bench_knobs_$i.log
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode > $D/bench_base.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $D/bench_base.log
