#!/bin/bash
# learner hyperparameters, round 2: long horizons (gamma -> 1) with the growth reward, and the stable knobs at a 1,000-step ramp
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 200 python tools/policy_breakdown.py --policies greedy --json $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^greedy' $O/$n.log | python -c "import sys,json; l=sys.stdin.read().split(' ',1)[1]; d=json.loads(l); print('$n', 'mean %.0f median %.0f corr %.3f shares %.1f zero %.3f' % (d['mean'], d['median'], d['pos_price_corr_median'], d['mean_shares'], d['zero_share_frac']))"
}
G="--set agent.reward_mode=growth"
run g0999_lr3e4 $G --set agent.gamma=0.999 --set agent.lr=0.0003
run g09995 $G --set agent.gamma=0.9995
run g0999_r300 $G --set agent.gamma=0.999 --set agent.ramp=300.0
run g0999_e05 $G --set agent.gamma=0.999 --set agent.epsilon=0.5
run r09995 --set agent.gamma=0.9995
run g0999_lr3e3 $G --set agent.gamma=0.999 --set agent.lr=0.003
run st_r1000_g --preset flagship_stable --set agent.ramp=1000.0 $G
run st_r500 --preset flagship_stable --set agent.ramp=500.0
run st_r1000_g0999 --preset flagship_stable --set agent.ramp=1000.0 --set agent.gamma=0.999
run g0999_t1000_dd $G --set agent.gamma=0.999 --set agent.target_every=1000 --set agent.double_dqn=true
