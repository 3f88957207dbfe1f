#!/bin/bash
# Tests (optional $TESTS) + 1-GPU bench + rocprofv3 kernel-trace stats of the flagship step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_k$i.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_k$i.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/kprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kprof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 > "$R/gpurun_out/kprof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/kprof.log"; exit $rc; }
cd "$R" && python tools/prof_summary.py $(find gpurun_out/kprof -name '*.db' | head -1) -o gpurun_out/kprof.md > /dev/null 2>&1; head -8 gpurun_out/kprof.md | cut -c1-200
