#!/bin/bash
# learning-rate sweep of the flagship learner at the 1M-env bench default (AR(1) bank, 3 episodes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sweep1m
i=0
while read -r line; do
  i=$((i+1))
  timeout -k 10 150 python tools/learning_curve.py --steps 17538 --envs 1048576 --every 5846 --kinds learned $line > gpurun_out/sweep1m/run$i.log 2>&1
  rc=$?; echo "== $i: $line"; grep '^learned' gpurun_out/sweep1m/run$i.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l.split(' ',1)[1]); print(d['step'], round(d['mean_reward']*1e4,3), round(d.get('final_portfolio_mean',0),1), '%.2e'%d['mean_td_loss'])" | tr '\n' ';'; echo
  [ $rc -eq 0 ] || exit $rc
done <<'LIST'
--set agent.lr=0.001
--set agent.lr=0.002
--set agent.lr=0.004
--set agent.lr=0.008
LIST
