#!/bin/bash
# full GPU suite (as the driver runs it) + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5full}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; grep -E "FAILED|ERROR" $D/pytest_gpu.log | head -20; tail -1 $D/pytest_gpu.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $D/smoke.log
