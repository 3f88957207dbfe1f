#!/bin/bash
# kernel statistics of the flagship bench and configs 4 / 5 on the final tree (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r5prof}
mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/flagship -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode > $D/flagship.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/deep -o run -- python3 benchmarks/bench_deep.py --steps 50 > $D/deep.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/gru -o run -- python3 benchmarks/bench_gru.py --steps 20 > $D/gru.log 2>&1 || exit 1
find $D -name "*kernel_stats.csv" | sort
