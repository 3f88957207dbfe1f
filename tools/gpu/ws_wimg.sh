#!/bin/bash
# ws weight images by LDS-DMA (kept current by the optimizer pass) vs the per-launch gather: GPU tests, kernel
# time at one chunk per workgroup, bench at the driver's arguments (A/B, 2 runs each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r5wimg}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_qstep_ws.py tests/test_gpu_ws_knobs.py tests/test_gpu_dp.py tests/test_gpu_eval.py tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for w in 0 1; do
  SHARETRADE_WS_WIMG=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/e16k_$w -o run -- python3 bench.py --envs 16384 --steps 40 --warmup 5 --no-episode > $D/e16k_$w.log 2>&1 || exit 1
  echo "wimg=$w 16384 envs: $(python3 tools/prof_summary.py $(find $D/e16k_$w -name '*.db' | head -1) | grep -E 'qstep_ws|reduce_optim' | cut -d'|' -f2-5 | tr '\n' ' ')"
done
for w in 0 1 0 1; do
  SHARETRADE_WS_WIMG=$w timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-episode > $D/bench_$w.log 2>&1 || exit 1
  echo "wimg=$w bench: $(grep -o '"ms_per_step": [0-9.]*' $D/bench_$w.log)"
done
