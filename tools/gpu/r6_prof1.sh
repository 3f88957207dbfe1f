#!/bin/bash
# kernel times of the plain and knob steps on the tick bank, the target-pass variants, then the learner sweep
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_plain -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode --no-graph > $O/plain.json 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_knobs -o run -- python3 bench.py --steps 20 --warmup 5 --no-episode --no-graph --target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global > $O/knobs.json 2> $O/knobs.err || { tail -20 $O/knobs.err; exit 1; }
find $O -name "*kernel_stats.csv" | head
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:6]: print(x['Name'][:90], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us')
"; done
timeout -k 10 200 python3 tools/bench_qtarget.py > $O/qtarget_variants.md 2>&1 || { tail -20 $O/qtarget_variants.md; exit 1; }
cat $O/qtarget_variants.md
bash tools/gpu/r6_sweep.sh
