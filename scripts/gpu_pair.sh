#!/bin/bash
# Pair-kernel check: its numerics tests, then interleaved bench A/B wide vs pair at 1M envs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -v --timeout 120 --timeout-method thread -k "pair or wide_and_narrow" > gpurun_out/pytest_pair.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_pair.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for k in wide pair; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --step-kernel $k > gpurun_out/bench_$k$i.log 2>&1
    rc=$?; echo "$k$i $(tail -1 gpurun_out/bench_$k$i.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
  done
done
