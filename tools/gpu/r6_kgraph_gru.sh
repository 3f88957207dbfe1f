#!/bin/bash
# config 5: k whole iterations per HIP graph -- tests, then A/B x3 (k = 1 vs 4)
set -o pipefail
O=gpurun_out/kgraph_gru
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gru.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
for i in 1 2 3; do
  for k in 1 4; do
    timeout -k 10 200 python -u benchmarks/bench_gru.py --steps 200 --iters-per-graph $k > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('k', d['iters_per_graph'], d.get('ms_per_iteration'), d.get('act_ms'), d.get('update_ms'))"
  done
done
tail -2 $O/tests.log
