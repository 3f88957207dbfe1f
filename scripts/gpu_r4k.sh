#!/bin/bash
# round 3: the driver's short bench window (20 steps after 5 warm-up) vs long windows, same box
set -o pipefail
mkdir -p gpurun_out
for a in "20 5" "20 5" "200 10" "20 5" "1000 100"; do
  set -- $a
  timeout -k 10 200 python -u bench.py --steps $1 --warmup $2 --no-episode > gpurun_out/r4k_$1_$2.log 2>&1 \
    || { echo BENCH_FAIL; tail -20 gpurun_out/r4k_$1_$2.log; exit 1; }
  echo "steps $1 warmup $2: $(tail -1 gpurun_out/r4k_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["graph_prime_steps"])')"
done
