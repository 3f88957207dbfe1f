#!/bin/bash
# flagship: kernel timeline of the captured multi-step graph (gaps between the step kernel and the optimizer pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/flagtl
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --steps 32 --warmup 5 --no-episode --no-stable-eval > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 40 -o $O/timeline.md > /dev/null || exit 1
head -44 $O/timeline.md
