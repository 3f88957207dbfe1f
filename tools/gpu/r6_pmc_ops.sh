#!/bin/bash
# torch.ops tests + the learner-median test, then PMC of the round-6 flagship step and the knob step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/r6m
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_torch_ops.py \
  "tests/test_gpu_eval.py::test_bench_learners_against_random_median" > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
grep -E "PASSED|FAILED|meas" $D/pytest.log
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES FETCH_SIZE --output-format csv -d $D/pmc1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-episode --no-graph > $D/pmc1.log 2>&1 || exit 1
f=$(find $D/pmc1 -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f --kernels qstep_ws,reduce_optim --title "PMC: round-6 flagship step (16-bit tick windows), 1,835,008 envs" -o $D/pmc_flagship.md && cat $D/pmc_flagship.md
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES FETCH_SIZE --output-format csv -d $D/pmc2 -o run -- python3 bench.py --steps 10 --warmup 3 --no-episode --no-graph --target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global > $D/pmc2.log 2>&1 || exit 1
f=$(find $D/pmc2 -name "*counter_collection.csv" | head -1)
python3 tools/pmc_summary.py $f --kernels qstep_ws,qtarget,reduce_optim --title "PMC: round-6 knob step (target pass variant 3, tick windows), 1,835,008 envs" -o $D/pmc_knobs.md && cat $D/pmc_knobs.md
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gru.py > $D/pytest_gru.log 2>&1 || { tail -40 $D/pytest_gru.log; exit 1; }
tail -1 $D/pytest_gru.log
for i in 1 2 3; do timeout -k 10 300 python benchmarks/bench_gru.py > $D/gru_$i.log 2>&1 || { tail -20 $D/gru_$i.log; exit 1; }; grep -E "ms|iteration" $D/gru_$i.log | tail -2; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_gru -o run -- python3 benchmarks/bench_gru.py --steps 20 > $D/prof_gru.log 2>&1 || exit 1
python3 tools/prof_summary.py $(find $D/prof_gru -name "*results.db" | head -1) | head -8
