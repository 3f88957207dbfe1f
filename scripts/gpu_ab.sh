#!/bin/bash
# A/B of step-kernel variants (csrc/qstep_wide8_<v>.hip): tests of the default build, alternating
# benches, then phase stamps of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
VARIANTS="${VARIANTS:-$(cat gpurun_variants.txt 2>/dev/null)}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in default $VARIANTS; do
    a=""; [ "$v" != default ] && a="--step-variant $v"
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 $a > gpurun_out/ab/bench_${v}_$i.log 2>&1
    rc=$?; echo "$v $i $(tail -1 gpurun_out/ab/bench_${v}_$i.log | cut -c100-125)"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in default $VARIANTS; do
  a=""; [ "$v" != default ] && a="--variant $v"
  timeout -k 10 120 python tools/stamp_qstep.py $a --out gpurun_out/ab/stamps_$v.md > gpurun_out/ab/stamps_$v.log 2>&1
  rc=$?; echo "== $v"; grep -E "P[0-9]|chunk loop \(|prologue|slab" gpurun_out/ab/stamps_$v.md | cut -d'|' -f2,3 | tr '\n' ';'; echo; [ $rc -eq 0 ] || exit $rc
done
