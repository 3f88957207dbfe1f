#!/bin/bash
# Round checkpoint: GPU suite, smoke, driver-style benches, 2-rank launch rehearsal, config 4, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ck
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ck/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/ck/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ck/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/ck/smoke.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ck/bench_20_5.log 2>&1
rc=$?; tail -1 gpurun_out/ck/bench_20_5.log | cut -c100-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/ck/bench_default.log 2>&1
rc=$?; tail -1 gpurun_out/ck/bench_default.log | cut -c100-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --envs 262144 --same-device --dist-backend gloo > gpurun_out/ck/rehearsal_n2.log 2>&1
rc=$?; grep -E '^\{' gpurun_out/ck/rehearsal_n2.log | cut -c100-220; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_deep.py > gpurun_out/ck/bench_deep.log 2>&1
rc=$?; tail -1 gpurun_out/ck/bench_deep.log | grep -oE '"ms_per_iteration": [0-9.]+|"env_steps_per_s": [0-9.]+|"updates_per_s": [0-9.]+' | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_gru.py > gpurun_out/ck/bench_gru.log 2>&1
rc=$?; tail -1 gpurun_out/ck/bench_gru.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ck/prof" -o run -- python3 "$R/bench.py" --steps 50 --warmup 10 > "$R/gpurun_out/ck/prof.log" 2>&1
rc=$?; tail -1 "$R/gpurun_out/ck/prof.log" | cut -c1-150; exit $rc
