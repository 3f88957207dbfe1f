#!/bin/bash
# the growth (2nd-order log) reward on the bench learner: greedy breakdown after the bench's 281 steps and longer
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python tools/policy_breakdown.py --policies greedy --json $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^greedy' $O/$n.log | sed "s/^/$n /"
}
run g09_281 --set agent.reward_mode=growth
run g099_281 --set agent.reward_mode=growth --set agent.gamma=0.99
run g09_1000 --set agent.reward_mode=growth --train-steps 1000
run rel09_1000 --train-steps 1000
run g097_281 --set agent.reward_mode=growth --set agent.gamma=0.97
