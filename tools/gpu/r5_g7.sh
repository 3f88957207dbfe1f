#!/bin/bash
# round 5: qtarget probe + reverted pipe kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5h}
mkdir -p $D
timeout -k 10 120 python -u tools/debug/qt_probe.py > $D/qt_probe.log 2>&1 || exit 1
cat $D/qt_probe.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py -v -s --timeout 120 --timeout-method thread -k "not dynamic" > $D/pytest_ws.log 2>&1
rc=$?; echo "ws+pipe pytest rc=$rc"; tail -1 $D/pytest_ws.log
