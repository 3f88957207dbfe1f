#!/bin/bash
# round 3: gradient waves form dZ2 (GDZ) -- numerics, A/B vs ddz (data waves form it) and gsingle, stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3z_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3z_ws.log; exit 1; }
tail -1 gpurun_out/r3z_ws.log
for rep in 1 2; do
for v in "" ddz gsingle; do
  extra="--step-kernel ws"; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode $extra > gpurun_out/r3z_bench_${v}_$rep.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r3z_bench_${v}_$rep.log; exit 1; }
  echo "$v $rep: $(tail -1 gpurun_out/r3z_bench_${v}_$rep.log | cut -c100-200)"
done
done
timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r3z_stamps_ws.md \
  > gpurun_out/r3z_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3z_stamps.log; exit 1; }
cat gpurun_out/r3z_stamps_ws.md
