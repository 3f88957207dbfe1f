#!/bin/bash
# round 3: ws kernel env-count sweep (bench.py --envs), 200 steps each
set -o pipefail
mkdir -p gpurun_out
for e in 65536 262144 1048576 1835008 3670016; do
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 10 --no-episode --envs $e > gpurun_out/r4l_$e.log 2>&1 \
    || { echo BENCH_FAIL $e; tail -20 gpurun_out/r4l_$e.log; exit 1; }
  echo "envs $e: $(tail -1 gpurun_out/r4l_$e.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], round(d["value"]/1e9,3), d.get("hbm_used_gb"))')"
done
