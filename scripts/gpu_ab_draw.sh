#!/bin/bash
# A/B: early epsilon-greedy draw (default) vs draw in P3 (variant nodraw): wide-kernel tests, stamps, benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qstep.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_qstep.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARS:-draw nodraw}; do
  vv=$v; [ "$v" = "draw" ] && vv=""
  timeout -k 10 120 python tools/stamp_qstep.py --envs 1048576 --variant "$vv" --out gpurun_out/stamps_$v.md > gpurun_out/stamps_$v.log 2>&1 || exit $?
  echo "== $v"; grep -E "P[0-9]|chunk loop \(" gpurun_out/stamps_$v.md | cut -c1-60
done
for i in 1 2; do
  for v in ${VARS:-draw nodraw}; do
    vv=$v; [ "$v" = "draw" ] && vv=""
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 --step-variant "$vv" > gpurun_out/bench_$v$i.log 2>&1 || exit $?
    echo "$v$i $(tail -1 gpurun_out/bench_$v$i.log | cut -c100-190)"
  done
done
