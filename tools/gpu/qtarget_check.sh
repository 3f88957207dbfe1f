#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5qt}
mkdir -p $D
timeout -k 10 200 python -u tools/bench_qtarget.py > $D/bench_qtarget.md 2>&1 || exit 1
grep "|" $D/bench_qtarget.md
timeout -k 10 300 python -u -m pytest tests/test_gpu_ws_knobs.py -q --timeout 120 --timeout-method thread > $D/pytest_knobs.log 2>&1
rc=$?; echo "knobs pytest rc=$rc"; tail -1 $D/pytest_knobs.log
