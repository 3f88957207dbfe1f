#!/bin/bash
# the stabilised learner at smaller batches (for a GPU test), and the bench with its stable-learner evaluation
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 200 python tools/policy_breakdown.py --json $O/$n.json "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep -E '^(greedy|random) ' $O/$n.log | python -c "
import sys,json
for line in sys.stdin:
    k,l=line.split(' ',1); d=json.loads(l)
    print('$n', k, 'mean %.0f median %.0f corr %.3f shares %.1f' % (d['mean'], d['median'], d['pos_price_corr_median'], d['mean_shares']))"
}
for E in 262144 524288; do
  run st500_$E --envs $E --preset flagship_stable --set agent.ramp=500.0 --policies greedy,random
  run plain_$E --envs $E --policies greedy
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench.py > $O/pytest_bench.log 2>&1 || { tail -30 $O/pytest_bench.log; exit 1; }
tail -2 $O/pytest_bench.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));e=d['episode_return'];print(d['ms_per_step'], {k:e[k] for k in ('greedy_median','random_median','buy_hold_median')}, e['stable_learner'])"
