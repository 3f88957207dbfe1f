#!/bin/bash
# Wide-chunk step kernel: numerics tests, 32- vs 64-env-chunk bench, phase stamps, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_qstep.log 2>&1
rc=$?; tail -25 gpurun_out/pytest_qstep.log; [ $rc -eq 0 ] || exit $rc
for c in 32 64; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --chunk $c > gpurun_out/bench_c$c.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_c$c.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python tools/stamp_qstep.py --chunk 64 --out gpurun_out/stamps64.md > gpurun_out/stamps64.log 2>&1
rc=$?; tail -14 gpurun_out/stamps64.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profw" -o run -- python3 "$R/bench.py" --steps 30 --warmup 5 --no-graph > "$R/gpurun_out/profw.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/profw.log"; exit $rc
