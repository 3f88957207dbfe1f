"""Debug: the 64-env-chunk kernel's bf16 column-blocked gradient slabs vs its fp32 row-major slabs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sharetrade.config import preset_config  # noqa: E402
from sharetrade.ops import native  # noqa: E402
from sharetrade.trainer.engine import VectorEngine  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 192
dev = torch.device("cuda", 0)
res = {}
for sd in ("fp32", "bf16"):
    cfg = preset_config("flagship")
    cfg.engine.chunk = 64
    cfg.engine.slab_dtype = sd
    eng = VectorEngine(cfg, device=dev, envs=E)
    eng.ctrl.fill_(5)
    eng.slab.fill_(float("nan"))
    L = native.lib()
    eng._launch_qstep(L, native.stream_handle())
    torch.cuda.synchronize()
    P, G = eng.layout.numel, eng.grid
    if sd == "fp32":
        slab = eng.slab.cpu().float()
    else:
        slab = eng.slab.cpu().float()[: P * G].view(P // 32, G, 32).permute(1, 0, 2).reshape(G, P)
    res[sd] = slab
    w = ~torch.isnan(slab)
    print(sd, "grid", G, "P", P, "written per row", w.sum(1).tolist(), "segments", {k: (v.offset, v.numel) for k, v in eng.layout.segments.items()})
s32, s16 = res["fp32"], res["bf16"]
w32, w16 = ~torch.isnan(s32), ~torch.isnan(s16)
print("written-mask equal", bool(torch.equal(w32, w16)), "only32", int((w32 & ~w16).sum()), "only16", int((w16 & ~w32).sum()))
both = w32 & w16
d = (s16 - s32).abs()[both]
print("max abs diff on both-written", float(d.max()), "max |s32|", float(s32[both].abs().max()))
bad = torch.zeros_like(w32)
bad[both] = (s16 - s32).abs()[both] > 1e-2 * float(s32[both].abs().max())
idx = torch.nonzero(bad)
print("bad", idx.shape[0], idx[:12].tolist())
raw = eng.slab.cpu().float()
print("raw[0:8]", raw[0:8].tolist())
print("raw[128:136]", raw[128:136].tolist())
print("raw[256:264]", raw[256:264].tolist())
print("raw[384:392]", raw[384:392].tolist())
for g in range(3):
    print("s32 row", g, s32[g, 0:8].tolist(), "cols128..", s32[g, 128:136].tolist())
