#!/bin/bash
# round 5: pipe kernel numerics vs the oracle, then a first timing of pipe and ws
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5b
timeout -k 10 420 python -u -m pytest tests/test_gpu_qstep_ws.py -v -s --timeout 120 --timeout-method thread -k "pipe and not dynamic" > gpurun_out/r5b/pytest_pipe.log 2>&1
echo "pytest rc=$?"
timeout -k 10 240 python -u bench.py --step-kernel pipe --steps 20 --warmup 5 --no-episode > gpurun_out/r5b/bench_pipe.log 2>&1 && \
timeout -k 10 240 python -u bench.py --step-kernel ws --steps 20 --warmup 5 --no-episode > gpurun_out/r5b/bench_ws.log 2>&1
rc=$?
tail -2 gpurun_out/r5b/bench_pipe.log gpurun_out/r5b/bench_ws.log
exit $rc
