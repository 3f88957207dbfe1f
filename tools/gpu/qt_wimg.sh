#!/bin/bash
# the target pass's weight images by LDS-DMA (refreshed with the target copy): knob tests, qtarget variants,
# knob step A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=gpurun_out/${TAG:-r5qtimg}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_ws_knobs.py tests/test_gpu_dp.py tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
K="--target-every 1000 --double-dqn --reward-scale 100 --ramp-mode global"
for w in 0 1 0 1; do
  SHARETRADE_WS_WIMG=$w timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-episode $K > $D/knobs_$w.log 2>&1 || exit 1
  echo "wimg=$w knob step: $(grep -o '"ms_per_step": [0-9.]*' $D/knobs_$w.log)"
done
