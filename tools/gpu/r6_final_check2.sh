#!/bin/bash
# final tree: deep + gemm GPU tests, config 4 / 5 defaults x3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu/r6_defaults45.sh
