#!/bin/bash
# 4-rank same-device gloo rehearsal of bench.py (split HIP graphs around the host-side all-reduce)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5g4}
mkdir -p $D
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 4 --dist-backend gloo --same-device --envs 131072 --steps 20 --warmup 5 --no-episode > $D/rehearsal_gloo4.log 2>&1 || exit 1
grep '^{' $D/rehearsal_gloo4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['ms_per_step'], d['config']['hip_graph'], d.get('alloc_peak_gb_per_rank'), d.get('allreduce_ms_per_step'))"
