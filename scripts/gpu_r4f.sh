#!/bin/bash
# round 3: checkpoint after fma / wbe -- GPU suite, default bench (driver args), production and gskipst stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4f_suite.log 2>&1 || { echo SUITE_FAIL; tail -60 gpurun_out/r4f_suite.log; exit 1; }
tail -1 gpurun_out/r4f_suite.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4f_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r4f_bench.log; exit 1; }
tail -1 gpurun_out/r4f_bench.log | cut -c1-400
for dv in "" gskipst; do
  timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --ws-dvariant "$dv" --out gpurun_out/r4f_stamps_ws$dv.md \
    > gpurun_out/r4f_stamps$dv.log 2>&1 || { echo STAMP_FAIL $dv; tail -30 gpurun_out/r4f_stamps$dv.log; exit 1; }
  cat gpurun_out/r4f_stamps_ws$dv.md
done
