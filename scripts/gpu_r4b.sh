#!/bin/bash
# round 3: learning curve at the bench batch (1,835,008 envs, ws kernel) + config-4 baseline with a kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u tools/learning_curve.py --steps 29230 --envs 1835008 --every 5846 \
  -o gpurun_out/r4b_learning.md > gpurun_out/r4b_learning.log 2>&1 || { echo LEARN_FAIL; tail -20 gpurun_out/r4b_learning.log; exit 1; }
cat gpurun_out/r4b_learning.md
timeout -k 10 200 python benchmarks/bench_deep.py > gpurun_out/r4b_deep.log 2>&1 || { echo DEEP_FAIL; tail -20 gpurun_out/r4b_deep.log; exit 1; }
tail -1 gpurun_out/r4b_deep.log | cut -c1-600
rm -rf gpurun_out/r4b_deepprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4b_deepprof" -o run -- python3 "$R/benchmarks/bench_deep.py" --steps 10 --warmup 8 > "$R/gpurun_out/r4b_deepprof.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/r4b_deepprof.log" | cut -c1-300; exit $rc
