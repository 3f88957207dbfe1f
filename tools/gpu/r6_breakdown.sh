#!/bin/bash
# the bench learner's greedy policy vs random / buy-and-hold / a fixed half-invested rule
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/policy_breakdown.py --out $O/breakdown_flagship.md --json $O/breakdown_flagship.json > $O/breakdown.log 2>&1 || { tail -30 $O/breakdown.log; exit 1; }
cat $O/breakdown_flagship.md
