#!/bin/bash
# GPU qstep tests + bench A/B of graph_steps (1 vs 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for g in 1 8; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 40 --graph-steps $g > gpurun_out/ab/bench_g${g}_$i.log 2>&1
    rc=$?; echo "g$g $i $(tail -1 gpurun_out/ab/bench_g${g}_$i.log | cut -c100-125)"; [ $rc -eq 0 ] || exit $rc
  done
done
