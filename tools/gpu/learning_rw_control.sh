#!/bin/bash
# learning knobs on the bench's own bank (random walk, no learnable signal), 262,144 envs
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5rw}
mkdir -p $D
ALL="agent.target_every=1000,agent.double_dqn=true,agent.reward_scale=100,agent.ramp_mode=global,agent.ramp=3000,agent.gamma=0.99"
timeout -k 10 600 python -u tools/learning_eval.py --envs 262144 --length 1601 --episodes 10 \
  --run "rw_base:data.source=random_walk" --run "rw_all:data.source=random_walk,$ALL" \
  -o $D/learning_rw.md > $D/learning.log 2>&1 || exit 1
tail -3 $D/learning.log
