#!/bin/bash
# round 3: ws stamps (data-wave build and gradient-wave build separately) + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode > gpurun_out/r3s_bench.log 2>&1 \
  || { echo BENCH_FAIL; tail -30 gpurun_out/r3s_bench.log; exit 1; }
echo "bench: $(tail -1 gpurun_out/r3s_bench.log | cut -c100-200)"
timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --out gpurun_out/r3s_stamps_ws.md \
  > gpurun_out/r3s_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3s_stamps.log; exit 1; }
cat gpurun_out/r3s_stamps_ws.md
timeout -k 10 60 python -u __graft_entry__.py smoke > gpurun_out/r3s_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/r3s_smoke.log; exit 1; }
tail -1 gpurun_out/r3s_smoke.log | cut -c1-200
