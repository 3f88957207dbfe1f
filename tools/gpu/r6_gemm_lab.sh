#!/bin/bash
# GEMM lab (timings, ablations, race screen), the production GEMM + deep-learner tests, the tile bench
# (vs hipBLASLt) and the config-4 bench
set -o pipefail
O=gpurun_out/lab
mkdir -p $O
timeout -k 10 200 tools/ubench/gemm_lab.bin > $O/lab.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_deep.py > $O/tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gemm_pp.py > $O/bench.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 200 >> $O/deep.log 2>&1 || exit 1; done
rc=$?
cat $O/lab.log; tail -3 $O/tests.log; cat $O/bench.log; grep -h "ms_per\|\"value\"" $O/deep.log | tail -6
exit $rc
