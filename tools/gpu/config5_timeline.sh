#!/bin/bash
# config 5 kernel timeline (bench_gru defaults)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5gru}
mkdir -p $D
timeout -k 10 300 python -u benchmarks/bench_gru.py > $D/bench_gru.log 2>&1 || exit 1
grep -o '"ms_per_iteration": [0-9.]*' $D/bench_gru.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/prof -o run -- python3 benchmarks/bench_gru.py --steps 10 > $D/prof.log 2>&1 || exit 1
f=$(find $D/prof -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 40 -o $D/timeline.md > /dev/null && head -50 $D/timeline.md
