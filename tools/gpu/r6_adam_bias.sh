#!/bin/bash
# config 4: Adam's bias reductions over 4-row blocks -- tests, Adam segment timings, bench x3
set -o pipefail
O=gpurun_out/adambias
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deep.py tests/test_gpu_learners_dp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/bench_adam_bias.py 2>&1 | grep "^|"
for i in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_deep.py > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('config4', d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
done
