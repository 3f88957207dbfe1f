#!/bin/bash
# the 16-bit tick windows: ws / knob / large-bank tests, then the bench (plain and with the learning knobs)
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_qstep_ws.py tests/test_gpu_ws_knobs.py \
  "tests/test_gpu_qstep.py::test_large_bank_gather_matches_oracle" > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -30; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-episode > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-episode --target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global > $O/bench_knobs.json 2> $O/bench_knobs.err || { tail -20 $O/bench_knobs.err; exit 1; }
cat $O/bench_knobs.json
