#!/bin/bash
# config 4: the hidden layers' Adam on its own stream (split_adam, new default) vs one launch at the join, A/B x3
# (historical record: the variant this A/B measured was removed afterwards, so its flag no longer exists)
set -o pipefail
O=gpurun_out/splitadam
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
for i in 1 2 3; do
  for g in split one; do
    f=""; [ $g = one ] && f="--no-split-adam"
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 200 $f > $O/$g.$i.json 2> $O/$g.$i.err || { tail $O/$g.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$g.$i.json')); print('$g', d['split_adam'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
grep -c PASSED $O/tests.log; tail -2 $O/tests.log
