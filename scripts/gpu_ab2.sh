#!/bin/bash
# full GPU suite + 3 benches + kernel-trace stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_all.log 2>&1
rc=$?; tail -1 gpurun_out/ab/pytest_all.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/ab/bench_$i.log 2>&1
  rc=$?; echo "$i $(tail -1 gpurun_out/ab/bench_$i.log | cut -c100-125)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/kprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kprof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 5 > "$R/gpurun_out/kprof.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/kprof.log"; exit $rc; }
cd "$R" && python tools/prof_summary.py $(find gpurun_out/kprof -name '*.db' | head -1) -o gpurun_out/kprof.md > /dev/null 2>&1; grep -E "qstep|reduce_optim" gpurun_out/kprof.md | cut -c1-160
