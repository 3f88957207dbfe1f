#!/bin/bash
# seed spread of the knob effect on the AR(1) bank (262,144 envs, 1,400-step episodes, 10 episodes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5seeds}
mkdir -p $D
ALL="agent.target_every=1000,agent.double_dqn=true,agent.reward_scale=100,agent.ramp_mode=global,agent.ramp=3000,agent.gamma=0.99"
R=""
for s in 1 2 3; do
  R="$R --run ar1_base_s$s:data.source=ar1,agent.seed=$s,data.seed=$s --run ar1_all_s$s:data.source=ar1,agent.seed=$s,data.seed=$s,$ALL"
done
timeout -k 10 1100 python -u tools/learning_eval.py --envs 262144 --length 1601 --episodes 10 $R \
  -o $D/learning_seeds.md 2>&1 | tee $D/learning.log
