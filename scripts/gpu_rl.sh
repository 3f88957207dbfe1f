#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_rl.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_rl$i.log 2>&1
rc=$?; tail -1 gpurun_out/bench_rl$i.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python tools/learning_curve.py --steps ${STEPS:-30000} --envs 65536 --every ${EVERY:-1000} -o gpurun_out/learning.md > gpurun_out/learning.log 2>&1
rc=$?; cat gpurun_out/learning.md; exit $rc
