#!/bin/bash
# configs 4 and 5 with default bench args (3 runs each), then a kernel timeline of each one's captured iterations
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/def45
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_deep.py > $O/deep_$i.json 2> $O/deep_$i.err || { tail $O/deep_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/deep_$i.json')); print('config4', d['ms_per_iteration'], d['act_ms'], d['update_ms'], d['iters_per_graph'])"
  timeout -k 10 200 python -u benchmarks/bench_gru.py > $O/gru_$i.json 2> $O/gru_$i.err || { tail $O/gru_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/gru_$i.json')); print('config5', d['ms_per_iteration'], d['act_ms'], d['update_ms'], d['iters_per_graph'])"
done
for w in gru deep; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$w -o run -- python3 tools/iter_only.py $w --iters 12 > $O/prof_$w.log 2>&1 || { tail $O/prof_$w.log; exit 1; }
  f=$(find $O/prof_$w -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 60 -o $O/timeline_$w.md > /dev/null || exit 1
done
head -70 $O/timeline_gru.md
