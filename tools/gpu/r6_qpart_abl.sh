#!/bin/bash
# config 4 kernel stats (round 6: run once with the EPI_BF16_QH head work compiled out by hand -- the qh flag forced
# false -- to price it: 25.9 vs 42.5 us before the qh_step fix, profiles/r6_config4_head.md)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qpabl
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/qf -o run -- python3 benchmarks/bench_deep.py --steps 64 > $O/qf.log 2>&1 || { tail $O/qf.log; exit 1; }
