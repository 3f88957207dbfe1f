#!/bin/bash
# target pass: next window position prefetched (variant 4) vs variant 3 -- per-launch bench, knob-step A/B x3
set -o pipefail
O=gpurun_out/qtpf
mkdir -p $O
timeout -k 10 200 python -u tools/bench_qtarget.py > $O/qt.log 2>&1 || { tail -20 $O/qt.log; exit 1; }
cat $O/qt.log
for i in 1 2 3; do
  for v in 3 4; do
    SHARETRADE_QT_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global --no-episode --no-stable-eval > $O/k$v.log 2>&1 || { tail $O/k$v.log; exit 1; }
    grep '^{' $O/k$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $v', d['ms_per_step'], d['value'])"
  done
done
