#!/bin/bash
# round 5: pipe kernel (interleaved phases, double-buffered LDS-DMA staging): numerics, timing, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5d}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py -v -s --timeout 120 --timeout-method thread -k "pipe and not dynamic" > $D/pytest_pipe.log 2>&1
echo "pytest rc=$?"; tail -1 $D/pytest_pipe.log
timeout -k 10 240 python -u bench.py --step-kernel pipe --steps 20 --warmup 5 --no-episode > $D/bench_pipe.log 2>&1 || exit 1
tail -1 $D/bench_pipe.log | cut -c1-300
SHARETRADE_AB_BUILDS=1 timeout -k 10 240 python -u tools/stamp_pipe.py --out $D/stamps_pipe.md > $D/stamps.log 2>&1 || exit 1
cat $D/stamps_pipe.md
