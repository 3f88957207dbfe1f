#!/bin/bash
# configs 4 and 5 with their benches' default arguments, 3 runs each
set -o pipefail
O=gpurun_out/def45
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_deep.py > $O/deep_$i.json 2> $O/deep_$i.err || { tail $O/deep_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/deep_$i.json')); print('config4', d['ms_per_iteration'], d['act_ms'], d['update_ms'], d['iters_per_graph'])"
  timeout -k 10 200 python -u benchmarks/bench_gru.py > $O/gru_$i.json 2> $O/gru_$i.err || { tail $O/gru_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/gru_$i.json')); print('config5', d['ms_per_iteration'], d['act_ms'], d['update_ms'], d['iters_per_graph'])"
done
