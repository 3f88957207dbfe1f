#!/bin/bash
# config 4: ring / step counters advanced in the env step's last block (no one-thread launch after it)
set -o pipefail
out=gpurun_out/${TAG:-r5c4a}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_learners_dp.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2 3; do
  timeout -k 10 150 python -u benchmarks/bench_deep.py --steps 200 > $out/deep_$i.json 2> $out/err.log || exit 1
  echo "run $i $(python -c "import json; d=json.loads(open('$out/deep_$i.json').read().splitlines()[-1]); print(d['ms_per_iteration'], d['update_ms'], d['act_ms'])")" | tee -a $out/summary.txt
done
