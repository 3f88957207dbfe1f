#!/bin/bash
# config 4: bench (3 runs) and one iteration's kernel timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/r6t
mkdir -p $D
for i in 1 2 3; do timeout -k 10 300 python -u benchmarks/bench_deep.py > $D/bench_deep_$i.log 2>&1 || { tail -20 $D/bench_deep_$i.log; exit 1; }; grep -o '"ms_per_iteration": [0-9.]*' $D/bench_deep_$i.log; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/prof -o run -- python3 benchmarks/bench_deep.py --steps 10 > $D/prof.log 2>&1 || exit 1
f=$(find $D/prof -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 40 -o $D/timeline.md > /dev/null && cat $D/timeline.md
