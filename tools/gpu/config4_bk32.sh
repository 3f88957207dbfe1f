#!/bin/bash
# config 4: 128x128 GEMMs with a 32-wide K tile and a 3- / 4-stage LDS ring vs BK 64 / 2 stages
set -o pipefail
out=gpurun_out/r5k32
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $out/pytest_gemm.log 2>&1 || { tail -30 $out/pytest_gemm.log; exit 1; }
tail -2 $out/pytest_gemm.log
timeout -k 10 120 python -u tools/bench_gemm_k32.py > $out/shapes.md 2>&1 || exit 1
cat $out/shapes.md
for v in "" s4 s3 "" s4 s3; do
  SHARETRADE_GEMM_BK32=$v timeout -k 10 150 python -u benchmarks/bench_deep.py --steps 200 > $out/deep_${v:-base}.json 2> $out/err.log || exit 1
  echo "bk32=${v:-base} $(python -c "import json; d=json.loads(open('$out/deep_${v:-base}.json').read().splitlines()[-1]); print(d['ms_per_iteration'], d['update_ms'], d['act_ms'])")" | tee -a $out/summary.txt
done
SHARETRADE_GEMM_BK32=s4 timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -x -q --timeout 120 --timeout-method thread > $out/pytest_deep_s4.log 2>&1; tail -2 $out/pytest_deep_s4.log
