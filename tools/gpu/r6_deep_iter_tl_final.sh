#!/bin/bash
# config 4: kernel timeline of the captured (overlapped) iterations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/tlfinal
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_deep2 -o run -- python3 tools/iter_only.py deep --iters 16 > $O/prof_deep2.log 2>&1 || { tail $O/prof_deep2.log; exit 1; }
f=$(find $O/prof_deep2 -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 40 -o $O/timeline_deep2.md > /dev/null || exit 1
head -3 $O/timeline_deep2.md
