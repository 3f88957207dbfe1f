#!/bin/bash
# round 3: data-wave stamps with the gradient waves idle (gskipst) -- how much of layer 1's in-situ time
# is the gradient waves' interference?
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/stamp_qstep.py --kernel ws --envs 1835008 --ws-dvariant gskipst --out gpurun_out/r3w_stamps_gskip.md \
  > gpurun_out/r3w_stamps.log 2>&1 || { echo STAMP_FAIL; tail -30 gpurun_out/r3w_stamps.log; exit 1; }
head -20 gpurun_out/r3w_stamps_gskip.md
