#!/bin/bash
# round 3 end: full GPU suite on the final tree + production vs pd10 on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4zz_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r4zz_suite.log; exit 1; }
tail -1 gpurun_out/r4zz_suite.log
for rep in 1 2; do
for v in "" pd10; do
  extra="--step-kernel ws"; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode $extra > gpurun_out/r4zz_bench_${v}_$rep.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r4zz_bench_${v}_$rep.log; exit 1; }
  echo "$v $rep: $(tail -1 gpurun_out/r4zz_bench_${v}_$rep.log | cut -c100-200)"
done
done
