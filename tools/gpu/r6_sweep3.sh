#!/bin/bash
# learner round 3: what in flagship_stable at a 500-step ramp beats random's median, and which parts are free
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 200 python tools/policy_breakdown.py --policies greedy --json $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^greedy' $O/$n.log | python -c "import sys,json; l=sys.stdin.read().split(' ',1)[1]; d=json.loads(l); print('$n', 'mean %.0f median %.0f corr %.3f shares %.1f zero %.3f' % (d['mean'], d['median'], d['pos_price_corr_median'], d['mean_shares'], d['zero_share_frac']))"
}
R="--set agent.ramp=500.0"
run rs100_g099_r500 $R --set agent.reward_scale=100.0 --set agent.gamma=0.99
run g099_r500 $R --set agent.gamma=0.99
run rs100_g09_r500 $R --set agent.reward_scale=100.0
run r500 $R
run st_r500_nodd --preset flagship_stable $R --set agent.double_dqn=false
run st_r500_pos --preset flagship_stable $R --set agent.ramp_mode=position
run st_r300 --preset flagship_stable --set agent.ramp=300.0
run st_r700 --preset flagship_stable --set agent.ramp=700.0
run st_r500_s1 --preset flagship_stable $R --set agent.seed=1
run st_r500_s2 --preset flagship_stable $R --set agent.seed=2
run g0999_r200 --set agent.reward_mode=growth --set agent.gamma=0.999 --set agent.ramp=200.0
run rs100_g099_r300 --set agent.ramp=300.0 --set agent.reward_scale=100.0 --set agent.gamma=0.99
