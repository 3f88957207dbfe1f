#!/bin/bash
# config 4: bias gradients from backward-epilogue partials -- tests, Adam timing, bench A/B x3
set -o pipefail
O=gpurun_out/bpart
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deep.py tests/test_gpu_learners_dp.py tests/test_gpu_gemm.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for f in "" "--no-bias-part"; do
    timeout -k 10 200 python -u benchmarks/bench_deep.py $f > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print('bias_part', d['bias_part'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
