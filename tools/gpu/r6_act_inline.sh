#!/bin/bash
# config 4: act step forked beside the backward (default) vs inline on the update's stream (no cross-queue edges),
# with the first act layer on our kernel (lib) or hipBLASLt (lib0); A/B x3 interleaved
set -o pipefail
O=gpurun_out/actinline
mkdir -p $O
for i in 1 2 3; do
  for g in fork inline inline0; do
    f=""; [ $g = inline ] && f="--act-inline"; [ $g = inline0 ] && f="--act-inline --act-gemm lib0"
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 200 $f > $O/$g.$i.json 2> $O/$g.$i.err || { tail $O/$g.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$g.$i.json')); print('$g', d['act_inline'], d['act_gemm'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
