#!/bin/bash
# config 4: act step layer 0 also on hipBLASLt (lib0) vs the 1024 -> 1024 layers only (lib, default), A/B x3
set -o pipefail
O=gpurun_out/actlib0
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
for i in 1 2 3; do
  for g in lib lib0; do
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 200 --act-gemm $g > $O/$g.$i.json 2> $O/$g.$i.err || { tail $O/$g.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$g.$i.json')); print('$g', d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
tail -2 $O/tests.log
