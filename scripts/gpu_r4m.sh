#!/bin/bash
# round 3: config-4 Adam with 8-entry bias blocks (all loads in flight) -- deep tests, bench, kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4m_deep_tests.log 2>&1 \
  || { echo DEEP_TEST_FAIL; tail -40 gpurun_out/r4m_deep_tests.log; exit 1; }
tail -1 gpurun_out/r4m_deep_tests.log
for r in 1 2; do
  timeout -k 10 200 python benchmarks/bench_deep.py > gpurun_out/r4m_deep_$r.log 2>&1 || { echo DEEP_FAIL; tail -20 gpurun_out/r4m_deep_$r.log; exit 1; }
  tail -1 gpurun_out/r4m_deep_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("iter", d["ms_per_iteration"], "act", d["act_ms"], "update", d["update_ms"])'
done
rm -rf gpurun_out/r4m_prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4m_prof" -o run -- python3 "$R/benchmarks/bench_deep.py" --steps 10 --warmup 8 > "$R/gpurun_out/r4m_prof.log" 2>&1
rc=$?; cd "$R"; [ $rc -eq 0 ] || { echo PROF_FAIL; exit $rc; }
python tools/prof_summary.py gpurun_out/r4m_prof/run_results.db | grep -E "adam|kernel \|"
