#!/bin/bash
# config 4: dW GEMM backend tests + A/B (HIP split-K vs hipBLASLt where faster)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/deepdw
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/deepdw/pytest.log 2>&1
rc=$?; tail -8 gpurun_out/deepdw/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in hip auto; do
    timeout -k 10 200 python benchmarks/bench_deep.py --dw-gemm $m > gpurun_out/deepdw/$m.$rep.log 2>&1 || exit $?
    echo "$m rep$rep $(tail -1 gpurun_out/deepdw/$m.$rep.log | cut -c1-400)"
  done
done
