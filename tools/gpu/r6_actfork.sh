#!/bin/bash
# config 4: act step forked after the update's forward (production) vs before it
set -o pipefail
O=gpurun_out/actfork
mkdir -p $O
for i in 1 2 3; do
  for f in "" "--act-before-fwd"; do
    timeout -k 10 200 python -u benchmarks/bench_deep.py $f > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('act_before_fwd' if '$f' else 'act_after_fwd', d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
