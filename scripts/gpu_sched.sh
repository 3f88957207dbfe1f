#!/bin/bash
# Dynamic chunk schedule: numerics tests, 1-GPU bench static vs dynamic, overlapped-DP rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sched.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sched.log; [ $rc -eq 0 ] || exit $rc
for s in static dynamic; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --chunk-schedule $s > gpurun_out/bench_$s.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_$s.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/overlap_rehearsal.py --steps 100 --usec 25 --cus 0,8,32,64 -o gpurun_out/overlap.md > gpurun_out/overlap.log 2>&1
rc=$?; cat gpurun_out/overlap.md; exit $rc
