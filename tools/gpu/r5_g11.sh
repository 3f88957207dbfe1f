#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5s}
mkdir -p $D
timeout -k 10 120 python -u tools/debug/qt_colprobe.py > $D/qt_colprobe.log 2>&1 || exit 1
grep -v amdgpu.ids $D/qt_colprobe.log | tail -3
timeout -k 10 300 python -u -m pytest tests/test_gpu_ws_knobs.py -v -s --timeout 120 --timeout-method thread > $D/pytest_knobs.log 2>&1
rc=$?; echo "knobs pytest rc=$rc"; tail -1 $D/pytest_knobs.log; grep "qtarget compat" $D/pytest_knobs.log
[ $rc -gt 1 ] && exit 1
K="--target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode $K > $D/bench_knobs.log 2>&1 || exit 1
grep '^{' $D/bench_knobs.log | cut -c150-260
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_knobs -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode $K > $D/prof_knobs.log 2>&1 || exit 1
f=$(find $D/prof_knobs -name "*kernel_stats.csv" | head -1); cut -d, -f1-6 $f | head -5
