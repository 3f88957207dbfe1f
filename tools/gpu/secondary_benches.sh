#!/bin/bash
# round-5 final tree: secondary benchmarks (configs 4 / 5, serving, fp32 reference net, the reference app)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5sec}
mkdir -p $D
timeout -k 10 300 python -u benchmarks/bench_deep.py > $D/bench_deep.log 2>&1 || exit 1
grep '^{' $D/bench_deep.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_gru.py > $D/bench_gru.log 2>&1 || exit 1
grep '^{' $D/bench_gru.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_serve.py > $D/bench_serve.log 2>&1 || exit 1
tail -3 $D/bench_serve.log | cut -c1-400
timeout -k 10 300 python -u benchmarks/bench_f32.py --envs 16384,65536 --paths batched,batched_det > $D/bench_f32.log 2>&1 || exit 1
tail -6 $D/bench_f32.log
timeout -k 10 600 python -u benchmarks/bench_app.py > $D/bench_app.log 2>&1 || exit 1
tail -3 $D/bench_app.log | cut -c1-400
