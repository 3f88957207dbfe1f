#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_dp.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --envs 16384 --dist-backend gloo --same-device > gpurun_out/bench_dp2.log 2>&1
rc=$?; grep -E "capture|Error" gpurun_out/bench_dp2.log | head -3; tail -1 gpurun_out/bench_dp2.log | cut -c1-300; exit $rc
