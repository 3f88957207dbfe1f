#!/bin/bash
# price the ws kernel's prologue: production vs the timing build that builds the weight images twice, at one
# 64-env chunk per workgroup (16,384 envs) and at the bench size
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export SHARETRADE_AB_BUILDS=1
D=gpurun_out/${TAG:-r5wspro}
mkdir -p $D
for e in 16384 1835008; do
  for v in "" pro2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/e${e}_${v:-prod} -o run -- python3 bench.py --envs $e --steps 40 --warmup 5 --no-episode ${v:+--step-variant $v} > $D/e${e}_${v:-prod}.log 2>&1 || exit 1
    echo "envs $e variant ${v:-prod}: $(python3 tools/prof_summary.py $(find $D/e${e}_${v:-prod} -name '*.db' | head -1) | grep -E 'qstep_ws' | cut -d'|' -f3-6)"
  done
done
