#!/bin/bash
# config 4: the act step env gather forked at the update start (early_env_gather) vs with its forward; tests, stats, A/B x3
# (historical record: the variant this A/B measured was removed afterwards, so its flag no longer exists)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/egath
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_deep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/qf -o run -- python3 benchmarks/bench_deep.py --steps 64 > $O/qf.log 2>&1 || { tail $O/qf.log; exit 1; }
for i in 1 2 3; do
  for g in qf gemm; do
    f=""; [ $g = gemm ] && f="--late-env-gather"
    timeout -k 10 200 python -u benchmarks/bench_deep.py --steps 256 $f > $O/$g.$i.json 2> $O/$g.$i.err || { tail $O/$g.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/$g.$i.json')); print('$g', d['early_env_gather'], d['ms_per_iteration'], d['act_ms'], d['update_ms'])"
  done
done
