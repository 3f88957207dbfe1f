#!/bin/bash
# flagship at the driver's arguments (--steps 20 --warmup 5): the 16-step graph + 4 single-step replays (default)
# vs one 20-step graph (--graph-steps 20), interleaved x3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gsteps
mkdir -p $O
for i in 1 2 3; do
  for g in 0 20; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --graph-steps $g > $O/b$g.$i.log 2>&1 || { tail $O/b$g.$i.log; exit 1; }
    grep '^{' $O/b$g.$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph_steps', d.get('graph_steps'), d['ms_per_step'], d['value'])"
  done
done
