#!/bin/bash
# full GPU suite + smoke + bench A/B of graph_steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_all.log 2>&1
rc=$?; tail -1 gpurun_out/ab/pytest_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/ab/smoke.log | cut -c1-100; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for g in ${GSTEPS:-8 16 32}; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 40 --graph-steps $g > gpurun_out/ab/bench_g${g}_$i.log 2>&1
    rc=$?; echo "g$g $i $(tail -1 gpurun_out/ab/bench_g${g}_$i.log | cut -c100-125)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 200 python bench.py > gpurun_out/ab/bench_default.log 2>&1
rc=$?; echo "default-cli $(tail -1 gpurun_out/ab/bench_default.log | cut -c100-160)"; exit $rc
