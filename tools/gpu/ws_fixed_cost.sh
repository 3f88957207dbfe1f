#!/bin/bash
# the ws step's per-launch fixed cost: kernel time at one 64-env chunk per workgroup (16,384 envs) and at two
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r5wsfix}
mkdir -p $D
for e in 16384 32768 65536; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/e$e -o run -- python3 bench.py --envs $e --steps 40 --warmup 5 --no-episode > $D/e$e.log 2>&1 || exit 1
  python3 tools/prof_summary.py $(find $D/e$e -name "*.db" | head -1) | grep -E "qstep_ws|reduce_optim" | cut -c1-160
done
