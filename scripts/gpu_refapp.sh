#!/bin/bash
# The reference application end to end (ShareTradeHelper: 10 workers x 5,846 steps, 203->200->3 net,
# AdaGrad, reference quirks) on the GPU, both engines; synthetic 6,047-day series (the MSFT file is
# not on the box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for e in vector actors; do
  timeout -k 10 500 python -m sharetrade train --preset reference_compat --engine $e --device cuda \
     --set data.source=random_walk > gpurun_out/refapp_$e.log 2>&1
  rc=$?; echo "== $e"; tail -n 1 gpurun_out/refapp_$e.log; [ $rc -eq 0 ] || exit $rc
done
