#!/bin/bash
# end-of-round check: the driver's bench invocation (twice), the full GPU suite, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5final}
mkdir -p $D
for i in 1 2; do
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_$i.log 2>&1 || exit 1
grep '^{' $D/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['episode_return']['greedy_mean'], d['episode_return']['buy_hold_mean'], d.get('alloc_peak_gb_per_rank'))"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; grep -E "FAILED|ERROR" $D/pytest_gpu.log | head; tail -1 $D/pytest_gpu.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $D/smoke.log | cut -c1-200
