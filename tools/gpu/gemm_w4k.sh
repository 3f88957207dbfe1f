#!/bin/bash
# 256x256 GEMM: 4 waves of 128x128 with a 5-stage ring of 32-wide K-tiles (w4k) vs ping-pong / w4 / hipBLASLt;
# then config 4 with w4k for the act step's layers
set -o pipefail
out=gpurun_out/r5w4k
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $out/pytest_gemm.log 2>&1 || { tail -30 $out/pytest_gemm.log; exit 1; }
tail -1 $out/pytest_gemm.log
timeout -k 10 200 python -u tools/bench_gemm_pp.py > $out/gemm.md 2>&1 || exit 1
cat $out/gemm.md
for v in pp w4k pp w4k; do
  SHARETRADE_GEMM_BIG=$v timeout -k 10 150 python -u benchmarks/bench_deep.py --steps 200 > $out/deep_$v.json 2> $out/err.log || exit 1
  echo "big=$v $(python -c "import json; d=json.loads(open('$out/deep_$v.json').read().splitlines()[-1]); print(d['ms_per_iteration'], d['update_ms'], d['act_ms'])")" | tee -a $out/summary.txt
done
