#!/bin/bash
# round 5: learning knobs on the flagship bf16 ws step (AR(1) / trend banks), and the 2-rank same-device gloo
# rehearsal of bench.py with split HIP graphs around the collective
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5g}
mkdir -p $D
ALL="agent.target_every=1000,agent.double_dqn=true,agent.reward_scale=100,agent.ramp_mode=global,agent.ramp=3000,agent.gamma=0.99"
timeout -k 10 420 python -u tools/learning_eval.py --envs ${LE_ENVS:-262144} --length 1601 --episodes ${LE_EPS:-20} \
  --run "ar1_base:data.source=ar1" --run "ar1_all:data.source=ar1,$ALL" \
  --run "trend_base:data.source=trend" --run "trend_all:data.source=trend,$ALL" \
  -o $D/learning_ws.md > $D/learning_ws.log 2>&1 || exit 1
tail -3 $D/learning_ws.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --dist-backend gloo --same-device --envs 262144 --steps 20 --warmup 5 --no-episode > $D/rehearsal_gloo2.log 2>&1 || exit 1
grep '^{' $D/rehearsal_gloo2.log | cut -c1-600
