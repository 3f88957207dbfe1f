#!/bin/bash
# Pair kernel: numerics tests, interval stamps, bench A/B vs wide.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread -k "pair" > gpurun_out/pytest_pair.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_pair.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamp_qstep.py --envs 1048576 --kernel pair --out gpurun_out/stamps_pair.md > gpurun_out/stamps_pair.log 2>&1
rc=$?; tail -16 gpurun_out/stamps_pair.log; [ $rc -eq 0 ] || exit $rc
for k in ${KERNELS:-pair wide}; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --step-kernel $k > gpurun_out/bench_$k.log 2>&1
  rc=$?; echo "$k $(tail -1 gpurun_out/bench_$k.log | cut -c100-200)"; [ $rc -eq 0 ] || exit $rc
done
