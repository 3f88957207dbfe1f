"""Kernel-time probe of csrc/optim.hip reduce_optim (run under rocprofv3 --kernel-trace --stats):
the flagship engine's slab pass in each mode, with and without the stats fold."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sharetrade.config import preset_config  # noqa: E402
from sharetrade.ops import native  # noqa: E402
from sharetrade.trainer.engine import VectorEngine  # noqa: E402

eng = VectorEngine(preset_config("flagship"), device=torch.device("cuda", 0), envs=65536)
eng.run(3)
L, sh = native.lib(), native.stream_handle()
for mode, stats in ((1, True), (2, True), (0, True), (0, False), (1, False)):
    o = native.OptimParams()
    C.pointer(o)[0] = eng._op
    o.mode = mode
    if not stats:
        o.stats = None
    # marker launches distinguish the groups in the trace
    for _ in range(mode + 1 + (0 if stats else 5)):
        native.check(L.st_advance(native.ptr(eng.ctrl), sh), "marker")
    for _ in range(30):
        native.check(L.st_reduce_optim(o, sh), "reduce")
    torch.cuda.synchronize()
print("done")
