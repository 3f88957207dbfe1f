#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qpabl
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/qf -o run -- python3 benchmarks/bench_deep.py --steps 64 > $O/qf.log 2>&1 || { tail $O/qf.log; exit 1; }
