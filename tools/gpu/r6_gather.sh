#!/bin/bash
# deep gather with 16-byte window loads: tests, config-4 bench x3, gather kernel times from a trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gather
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_deep.py > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('config4', d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 tools/iter_only.py deep --iters 12 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name "*.db" | head -1); python3 tools/prof_timeline.py $f --last 60 -o $O/timeline.md > /dev/null || exit 1
grep gather $O/timeline.md | head -8
