#!/bin/bash
# round 3: where the step's time goes under the bench (HIP graphs, no counters): kernel trace timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r3r_trace
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d "$R/gpurun_out/r3r_trace" -o run -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-episode > "$R/gpurun_out/r3r_trace.log" 2>&1
rc=$?; tail -1 "$R/gpurun_out/r3r_trace.log" | cut -c100-200; [ $rc -eq 0 ] || exit $rc
cd "$R"
db=$(find gpurun_out/r3r_trace -name '*.db' | head -1)
python tools/prof_timeline.py "$db" --last 24 --title "bench.py (HIP graphs, 1,835,008 envs): last 24 kernels" -o gpurun_out/r3r_timeline.md && cat gpurun_out/r3r_timeline.md
