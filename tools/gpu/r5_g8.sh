#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5i}
mkdir -p $D
timeout -k 10 120 python -u tools/debug/qt_colprobe.py > $D/qt_colprobe.log 2>&1 || exit 1
grep -v amdgpu.ids $D/qt_colprobe.log | tail -8
timeout -k 10 120 python -u tools/debug/qt_probe.py > $D/qt_probe.log 2>&1 || exit 1
grep "rel=" $D/qt_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ws_knobs.py -v -s --timeout 120 --timeout-method thread > $D/pytest_knobs.log 2>&1
rc=$?; echo "knobs pytest rc=$rc"; tail -1 $D/pytest_knobs.log
