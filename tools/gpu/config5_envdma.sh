#!/bin/bash
# config 5: the env phase's next-step prefetch by LDS-DMA into the parked env state (no HBM wait in the
# env phase) -- GRU GPU tests, then bench_gru x3
set -o pipefail
out=gpurun_out/${TAG:-r5c5d}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py -x -q --timeout 120 --timeout-method thread > $out/pytest_gru.log 2>&1 || { tail -30 $out/pytest_gru.log; exit 1; }
tail -1 $out/pytest_gru.log
for i in 1 2 3; do
  timeout -k 10 150 python -u benchmarks/bench_gru.py > $out/gru_$i.json 2> $out/err.log || exit 1
  echo "run $i $(python -c "import json; d=json.loads(open('$out/gru_$i.json').read().splitlines()[-1]); print(d['ms_per_iteration'], d['act_ms'], d['update_ms'], d['env_steps_per_s'])")" | tee -a $out/summary.txt
done
