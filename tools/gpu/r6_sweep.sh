#!/bin/bash
# learner hyperparameters at the bench's batch and 281 steps: greedy median vs random's 216
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 200 python tools/policy_breakdown.py --policies greedy --json $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^greedy' $O/$n.log | python -c "import sys,json; l=sys.stdin.read().split(' ',1)[1]; d=json.loads(l); print('$n', 'mean %.0f median %.0f corr %.3f shares %.1f zero %.3f' % (d['mean'], d['median'], d['pos_price_corr_median'], d['mean_shares'], d['zero_share_frac']))"
}
run stable --preset flagship_stable
run stable_g --preset flagship_stable --set agent.reward_mode=growth
run stable_r1000 --preset flagship_stable --set agent.ramp=1000.0
run g0999 --set agent.reward_mode=growth --set agent.gamma=0.999
run r0999 --set agent.gamma=0.999
run r099 --set agent.gamma=0.99
run g099_lr3e4 --set agent.reward_mode=growth --set agent.gamma=0.99 --set agent.lr=0.0003
run g099_lr3e3 --set agent.reward_mode=growth --set agent.gamma=0.99 --set agent.lr=0.003
run t100_dd --set agent.target_every=100 --set agent.double_dqn=true --set agent.gamma=0.99
run t100_dd_g --set agent.target_every=100 --set agent.double_dqn=true --set agent.gamma=0.99 --set agent.reward_mode=growth
