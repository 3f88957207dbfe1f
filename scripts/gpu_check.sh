#!/bin/bash
# One gpurun call: build, GPU tests, short bench, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-100} --warmup 10 > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --no-graph > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit $rc
fi
