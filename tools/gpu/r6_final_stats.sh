#!/bin/bash
# final tree: rocprofv3 kernel stats of the flagship step, config 4 and config 5 benches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/finalstats
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/flag -o run -- python3 bench.py --steps 40 --warmup 5 --no-episode --no-stable-eval > $O/flag.log 2>&1 || { tail $O/flag.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/deep -o run -- python3 benchmarks/bench_deep.py --steps 50 > $O/deep.log 2>&1 || { tail $O/deep.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gru -o run -- python3 benchmarks/bench_gru.py --steps 50 > $O/gru.log 2>&1 || { tail $O/gru.log; exit 1; }
find $O -name "*kernel_stats.csv" | head
