#!/bin/bash
# Tuning sweep: phase stamps + 1-GPU bench for each kernel variant in $VARIANTS ("" = default build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
python build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
for v in ${VARIANTS:-w8}; do
  vv=$v; [ "$v" = "w8" ] && vv=""
  timeout -k 10 120 python tools/stamp_qstep.py --variant "$vv" --out gpurun_out/stamps_$v.md > gpurun_out/stamps_$v.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py --steps ${STEPS:-300} --warmup 30 --step-variant "$vv" > gpurun_out/bench_$v.log 2>&1 || exit $?
  echo "== $v"; grep -E "P[0-9]|chunk loop \(" gpurun_out/stamps_$v.md | cut -c1-60
  tail -1 gpurun_out/bench_$v.log | cut -c1-140
done
