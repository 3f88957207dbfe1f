#!/bin/bash
# round 3: gradient-wave fragment order A/B (production latency order vs the v4 order "gold", X 1 ahead "gx1")
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3q_ws.log 2>&1 || { echo WS_FAIL; tail -60 gpurun_out/r3q_ws.log; exit 1; }
tail -1 gpurun_out/r3q_ws.log
for rep in 1 2; do
for v in "" gold gx1; do
  extra="--step-kernel ws"; [ -n "$v" ] && extra="--step-kernel ws --step-variant $v"
  timeout -k 10 150 python -u bench.py --steps 200 --warmup 10 --no-episode $extra > gpurun_out/r3q_bench_${v}_$rep.log 2>&1 \
    || { echo BENCH_FAIL $v; tail -30 gpurun_out/r3q_bench_${v}_$rep.log; exit 1; }
  echo "$v $rep: $(tail -1 gpurun_out/r3q_bench_${v}_$rep.log | cut -c100-200)"
done
done
# round 3: where the step's time goes under the bench (HIP graphs, no counters): kernel trace timeline
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
R=$(pwd)
rm -rf gpurun_out/r3r_trace
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d "$R/gpurun_out/r3r_trace" -o run -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-episode > "$R/gpurun_out/r3r_trace.log" 2>&1
rc=$?; tail -1 "$R/gpurun_out/r3r_trace.log" | cut -c100-200; [ $rc -eq 0 ] || exit $rc
cd "$R"
db=$(find gpurun_out/r3r_trace -name '*.db' | head -1)
python tools/prof_timeline.py "$db" --last 24 --title "bench.py (HIP graphs, 1,835,008 envs): last 24 kernels" -o gpurun_out/r3r_timeline.md && cat gpurun_out/r3r_timeline.md
