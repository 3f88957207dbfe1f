#!/bin/bash
# config 4: fused TD + output-layer backward (deep_head_kernel) -- tests, then A/B x3
set -o pipefail
O=gpurun_out/head
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deep.py tests/test_gpu_learners_dp.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
for i in 1 2 3; do
  for f in "" "--no-fuse-head"; do
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 200 $f > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('fuse_head', d['fuse_head'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
tail -2 $O/tests.log
