#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5v}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -v -s --timeout 240 --timeout-method thread > $D/pytest_dp.log 2>&1
rc=$?; echo "dp pytest rc=$rc"; grep "PASSED\|FAILED\|Error" $D/pytest_dp.log | head -20; tail -1 $D/pytest_dp.log
