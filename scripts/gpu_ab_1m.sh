#!/bin/bash
# A/B of step-kernel launch options at the 1M-env default (same box, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab1m
for rep in 1 2; do
  for v in "default:" "dynamic:--chunk-schedule dynamic" "waves4:--step-waves 4" "gs4:--graph-steps 4"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 120 python bench.py --steps 500 --warmup 50 $a > gpurun_out/ab1m/$n.$rep.log 2>&1 || exit $?
    echo "$n rep$rep $(tail -1 gpurun_out/ab1m/$n.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"]/1e9, d["ms_per_step"])')"
  done
done
