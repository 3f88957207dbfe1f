#!/bin/bash
# config 4: per-layer Adam beside the backward chain (layer_adam) -- tests and A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
D=gpurun_out/${TAG:-r5x}
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py -v --timeout 240 --timeout-method thread > $D/pytest_deep.log 2>&1
rc=$?; echo "deep pytest rc=$rc"; grep -E "FAILED" $D/pytest_deep.log | head; tail -1 $D/pytest_deep.log
[ $rc -gt 1 ] && exit 1
for i in 1 2; do
  for la in 1 0; do
    SHARETRADE_DEEP_LAYER_ADAM=$la timeout -k 10 200 python -u benchmarks/bench_deep.py > $D/bench_deep_la${la}_$i.log 2>&1 || exit 1
    echo "layer_adam=$la: $(grep -o "\"ms_per_iteration[^,]*" $D/bench_deep_la${la}_$i.log | head -1) $(grep -o '"act_ms[^,]*' $D/bench_deep_la${la}_$i.log | head -1) $(grep -o '"update_ms[^,]*' $D/bench_deep_la${la}_$i.log | head -1)"
  done
done
