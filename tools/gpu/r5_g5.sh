#!/bin/bash
# round 5: ws learning knobs (target net / Double DQN / reward scale / global ramp) vs the oracle, then the
# pipe kernel (numerics, timing, stamps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5f}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_ws_knobs.py -v -s --timeout 120 --timeout-method thread > $D/pytest_knobs.log 2>&1
rc=$?; echo "knobs pytest rc=$rc"; tail -1 $D/pytest_knobs.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_dp_router_f32.py -v -s --timeout 240 --timeout-method thread -k "split_partials or rank_death or knobs" > $D/pytest_f32.log 2>&1
rc=$?; echo "f32 pytest rc=$rc"; tail -1 $D/pytest_f32.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 200 python -u benchmarks/bench_f32.py --envs 16384,65536 --paths batched,batched_det --steps 50 --out $D/bench_f32_det.md > $D/bench_f32.log 2>&1 || exit 1
tail -4 $D/bench_f32.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep_ws.py -v -s --timeout 120 --timeout-method thread -k "pipe and not dynamic" > $D/pytest_pipe.log 2>&1
rc=$?; echo "pipe pytest rc=$rc"; tail -1 $D/pytest_pipe.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 240 python -u bench.py --step-kernel pipe --steps 20 --warmup 5 --no-episode > $D/bench_pipe.log 2>&1 || exit 1
tail -1 $D/bench_pipe.log | cut -c1-300
SHARETRADE_AB_BUILDS=1 timeout -k 10 240 python -u tools/stamp_pipe.py --out $D/stamps_pipe.md > $D/stamps.log 2>&1 || exit 1
cat $D/stamps_pipe.md
