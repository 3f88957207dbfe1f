#!/bin/bash
# learning knobs on the flagship ws kernel at the bench's exact shape: 1,835,008 envs, 6,047-day series
# (5,846-step episodes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5fs}
mkdir -p $D
ALL="agent.target_every=1000,agent.double_dqn=true,agent.reward_scale=100,agent.ramp_mode=global,agent.ramp=3000,agent.gamma=0.99"
timeout -k 10 1100 python -u tools/learning_eval.py --envs 1835008 --length 6047 --episodes 3 \
  --run "ar1_base:data.source=ar1" --run "ar1_all:data.source=ar1,$ALL" \
  --run "trend_base:data.source=trend" --run "trend_all:data.source=trend,$ALL" \
  -o $D/learning_full_series.md 2>&1 | tee $D/learning.log
