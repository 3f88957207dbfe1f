#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5r}
mkdir -p $D
K="--target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_knobs -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode $K > $D/prof_knobs.log 2>&1 || exit 1
f=$(find $D/prof_knobs -name "*kernel_stats.csv" | head -1); echo $f; cut -d, -f1-8 $f | head -12
