#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sweep
i=0
while read -r line; do
  i=$((i+1))
  timeout -k 10 120 python tools/learning_curve.py --steps 30000 --envs 65536 --every 5846 --kinds learned $line > gpurun_out/sweep/run$i.log 2>&1
  rc=$?; echo "== $i: $line"; grep '^learned' gpurun_out/sweep/run$i.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l.split(' ',1)[1]); print(d['step'], round(d['mean_reward']*1e4,3), round(d.get('final_portfolio_mean',0),1), '%.2e'%d['mean_td_loss'])" | tr '\n' ';'; echo
  [ $rc -eq 0 ] || exit $rc
done <<'LIST'
--kinds random
--set agent.gamma=0.99
--set agent.gamma=0.9
--set agent.gamma=0.9 --set agent.lr=0.0003
--set agent.gamma=0.5
--set agent.gamma=0.99 --set agent.lr=0.0001
--set agent.gamma=0.9 --set agent.td_clip=1.0
LIST
