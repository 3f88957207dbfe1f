#!/bin/bash
# learned-policy sweep at the bench batch (1,835,008 envs, ws kernel): 3 episodes per setting
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r4c
i=0
while read -r line; do
  i=$((i+1))
  echo "== $i: $line"
  timeout -k 10 150 python tools/learning_curve.py --steps 17538 --envs 1835008 --every 5846 --kinds learned $line \
    -o gpurun_out/r4c/run$i.md > gpurun_out/r4c/run$i.log 2>&1 || { echo FAIL; tail -5 gpurun_out/r4c/run$i.log; exit 1; }
  grep "^| [0-9]" gpurun_out/r4c/run$i.md | awk -F'|' '{printf "%s %s %s %s;", $2, $3, $6, $9}'; echo
done <<'LIST'
--set agent.lr=0.0003
--set agent.lr=0.003
--set agent.gamma=0.5
--set agent.gamma=0.0
--set agent.gamma=0.5 --set agent.lr=0.0003
--set agent.epsilon=0.98
LIST
