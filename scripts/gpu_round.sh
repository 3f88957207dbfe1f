#!/bin/bash
# Round check: GPU suite + smoke + the driver's bench invocation (20/5) + default bench + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_20_5.log 2>&1
rc=$?; tail -1 gpurun_out/bench_20_5.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -1 gpurun_out/bench_default.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 10 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/prof.log" | cut -c1-300; exit $rc
