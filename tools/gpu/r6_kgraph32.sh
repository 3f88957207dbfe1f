#!/bin/bash
# config 4 and config 5: iterations per graph launch 16 (default) vs 32, interleaved x3
set -o pipefail
O=gpurun_out/kg32
mkdir -p $O
for i in 1 2 3; do
  for k in 16 32; do
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 512 --iters-per-graph $k > $O/d$k.$i.json 2> $O/d$k.$i.err || { tail $O/d$k.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/d$k.$i.json')); print('deep', d['iters_per_graph'], d['ms_per_iteration'])"
  done
done
for i in 1 2 3; do
  for k in 16 32; do
    timeout -k 10 200 python -u benchmarks/bench_gru.py --steps 256 --iters-per-graph $k > $O/g$k.$i.json 2> $O/g$k.$i.err || { tail $O/g$k.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/g$k.$i.json')); print('gru', d['iters_per_graph'], d.get('ms_per_iteration', d.get('ms_per_step')))"
  done
done
