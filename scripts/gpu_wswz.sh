#!/bin/bash
# A/B: default 8-wave step kernel vs the wswz tuning build (tests, stamps, interleaved benches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wswz
timeout -k 10 200 python -u -m pytest tests/test_gpu_qstep.py -x -q --timeout 120 --timeout-method thread -k "wswz or matches_oracle" > gpurun_out/wswz/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/wswz/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "" wswz; do
  timeout -k 10 120 python tools/stamp_qstep.py --variant "$v" --out gpurun_out/wswz/stamps_${v:-default}.md > gpurun_out/wswz/stamps_${v:-default}.log 2>&1 || exit $?
  grep -E "P[0-9]|chunk loop \(" gpurun_out/wswz/stamps_${v:-default}.md | cut -c1-60
done
for rep in 1 2; do
  for v in "" wswz; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 30 --step-variant "$v" > gpurun_out/wswz/bench_${v:-default}_$rep.log 2>&1 || exit $?
    echo "${v:-default} $rep $(tail -1 gpurun_out/wswz/bench_${v:-default}_$rep.log | cut -c100-190)"
  done
done
