#!/bin/bash
# final tree: rocprofv3 kernel stats of config 4 (after the folded output head)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/finalstats2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/deep -o run -- python3 benchmarks/bench_deep.py --steps 128 > $O/deep.log 2>&1 || { tail $O/deep.log; exit 1; }
grep -o '"ms_per_iteration": [0-9.]*' $O/deep.log
