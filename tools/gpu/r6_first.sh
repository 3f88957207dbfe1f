#!/bin/bash
# round 6, first box: the changed GPU tests, the driver's bench arguments, the window-gather ubench (+ aligned u16)
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_f32.py::test_fp32_batched_deterministic_wide_layers" \
  "tests/test_gpu_qstep_ws.py::test_ws_weight_image_stays_equal_to_fresh_pack" \
  "tests/test_gpu_ws_knobs.py::test_other_bf16_kernels_refuse_the_knobs" \
  "tests/test_gpu_dp.py::test_overlapped_dp_with_target_net_is_rank_consistent" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 tools/ubench/window_gather.bin 1835008 same 0 > $O/gather_same.md 2>&1 || exit 1
cat $O/gather_same.md
