#!/bin/bash
# round 5, GPU call 1: the new pipe kernel's numerics vs the oracle (and ws), then a first timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5a
timeout -k 10 420 python -u -m pytest tests/test_gpu_qstep_ws.py -x -v -s --timeout 120 --timeout-method thread -k "not dynamic" > gpurun_out/r5a/pytest_ws.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py --step-kernel pipe --steps 20 --warmup 5 --no-episode > gpurun_out/r5a/bench_pipe.log 2>&1 && \
timeout -k 10 240 python -u bench.py --step-kernel ws --steps 20 --warmup 5 --no-episode > gpurun_out/r5a/bench_ws.log 2>&1
rc=$?
tail -2 gpurun_out/r5a/bench_pipe.log gpurun_out/r5a/bench_ws.log
exit $rc
