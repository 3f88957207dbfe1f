#!/bin/bash
# A/B of ws step-kernel builds: the ws oracle tests on each variant, then interleaved bench runs
# usage: bash tools/gpu/ab_ws.sh OUTDIR "variant1 variant2 ..." [bench reps]
set -o pipefail
O=$1; VARS=$2; REPS=${3:-2}
mkdir -p $O
export PYTHONUNBUFFERED=1 SHARETRADE_AB_BUILDS=1
for v in $VARS; do
  SHARETRADE_WS_VARIANT=$v timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_qstep_ws.py -k "matches_oracle or tick_bank or trajectory" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for r in $(seq 1 $REPS); do
  for v in base $VARS; do
    a=""; [ "$v" != "base" ] && a="--step-variant $v"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-episode $a > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -20 $O/bench_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v rep $r', d['ms_per_step'])"
  done
done
