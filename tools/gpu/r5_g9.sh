#!/bin/bash
# round 5: cost of the learning knobs at the bench batch (ws default vs target net + Double DQN + ...), kernel
# stats of the knob run, and the AR(1) greedy-vs-random test on the flagship kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5q}
mkdir -p $D
K="--target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode > $D/bench_base.log 2>&1 || exit 1
grep '^{' $D/bench_base.log | cut -c1-260
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode $K > $D/bench_knobs.log 2>&1 || exit 1
grep '^{' $D/bench_knobs.log | cut -c1-260
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-episode > $D/bench_base2.log 2>&1 || exit 1
grep '^{' $D/bench_base2.log | cut -c1-260
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_knobs -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode $K > $D/prof_knobs.log 2>&1 || exit 1
find $D/prof_knobs -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py -v -s --timeout 240 --timeout-method thread -k "greedy" > $D/pytest_eval.log 2>&1
rc=$?; echo "eval pytest rc=$rc"; grep "\[meas\]\|passed\|failed" $D/pytest_eval.log | tail -4
