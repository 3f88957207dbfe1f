#!/bin/bash
# Quick perf loop: build, phase stamps of the 64-env-chunk kernel, 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python tools/stamp_qstep.py --chunk ${CHUNK:-64} --out gpurun_out/stamps.md > gpurun_out/stamps.log 2>&1
rc=$?; tail -16 gpurun_out/stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --chunk ${CHUNK:-64} > gpurun_out/bench_quick.log 2>&1
rc=$?; tail -1 gpurun_out/bench_quick.log | cut -c1-330; exit $rc
