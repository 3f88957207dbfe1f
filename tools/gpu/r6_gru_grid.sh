#!/bin/bash
# config 5: actor grid sweep (auto = 205 on 256 CUs: 5 rounds of chunk pairs)
set -o pipefail
O=gpurun_out/grugrid
mkdir -p $O
for g in 0 256 228 171; do
  for i in 1 2; do
    timeout -k 10 200 python -u benchmarks/bench_gru.py --grid $g > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('grid', d['actor_grid'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
