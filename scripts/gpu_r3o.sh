#!/bin/bash
# round 3: GPU rehearsals of the multi-rank control planes on one card (gloo, every rank on cuda:0):
# (1) the router fan-out as the DP plane: the reference app (train --engine vector) on 2 ranks over the
#     full MSFT series, one rank killed mid-episode -> routee replaced, group respawned, resumed;
# (2) the elastic engine CLI: 2 ranks, a rank killed at step 300 -> generation respawned from the last
#     committed shards, same final parameters as an uninterrupted run.
set -o pipefail
mkdir -p gpurun_out/r3o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m sharetrade train --preset intended --engine vector --gpus 2 --same-device \
  --dist-backend gloo --envs-per-rank 64 --ckpt-dir gpurun_out/r3o/dp_ckpt --ckpt-every 500 \
  > gpurun_out/r3o/dp_clean.log 2>&1 || { echo DP_CLEAN_FAIL; tail -40 gpurun_out/r3o/dp_clean.log; exit 1; }
tail -3 gpurun_out/r3o/dp_clean.log
SHARETRADE_FAIL_AT=1:1200:0 timeout -k 10 300 python -u -m sharetrade train --preset intended --engine vector --gpus 2 \
  --same-device --dist-backend gloo --envs-per-rank 64 --ckpt-dir gpurun_out/r3o/dp_ckpt_fail --ckpt-every 500 \
  > gpurun_out/r3o/dp_fail.log 2>&1 || { echo DP_FAIL_FAIL; tail -40 gpurun_out/r3o/dp_fail.log; exit 1; }
tail -3 gpurun_out/r3o/dp_fail.log
for tag in clean fail; do
  extra=""; [ $tag = fail ] && export SHARETRADE_FAIL_AT=1:300:0
  timeout -k 10 300 python -u -m sharetrade engine --preset flagship --elastic 2 --same-device --dist-backend gloo \
    --steps 600 --envs 65536 --ckpt-dir gpurun_out/r3o/el_$tag/ckpt --ckpt-every 200 --final-dir gpurun_out/r3o/el_$tag/final \
    --log-every 0 --stall-timeout 60 > gpurun_out/r3o/el_$tag.log 2>&1 || { echo EL_FAIL $tag; tail -40 gpurun_out/r3o/el_$tag.log; exit 1; }
  unset SHARETRADE_FAIL_AT
  tail -1 gpurun_out/r3o/el_$tag.log | cut -c1-400
done
python - <<'PY'
import torch
from sharetrade.persist import checkpoint as ck
a = [ck.load(f"gpurun_out/r3o/el_{t}/final/final-rank-0.stck")[0] for t in ("clean", "fail")]
print("elastic final params bit-identical after a rank death:", torch.equal(a[0]["params"], a[1]["params"]),
      "steps", int(a[0]["step"][0]), int(a[1]["step"][0]))
PY
rm -rf gpurun_out/r3o/*ckpt* gpurun_out/r3o/el_*/ckpt
