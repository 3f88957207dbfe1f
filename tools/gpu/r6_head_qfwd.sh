#!/bin/bash
# config 4: the output layer's forward inside deep_head_kernel (head_qfwd, new default) vs the batched split-K
# output GEMM; GPU tests, then A/B x3 interleaved
set -o pipefail
O=gpurun_out/headq
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log
for i in 1 2 3; do
  for g in qf gemm; do
    f=""; [ $g = gemm ] && f="--no-head-qfwd"
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 256 $f > $O/$g.$i.json 2> $O/$g.$i.err || { tail $O/$g.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$g.$i.json')); print('$g', d['head_qfwd'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
