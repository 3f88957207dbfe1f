"""Hidden-unit probe of csrc/qtarget.hip: h1[u] = (u + 1) / 128 (through the constant input column), layer 2 a
permutation sigma, the output row 0 = e_v: QT[.][.][0] must be h1[sigma^-1(v)] (and with W0 = 0, relu(b1[v]))."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from test_gpu_qstep_ws import _cfg, _prices  # noqa: E402

from sharetrade.ops import native  # noqa: E402
from sharetrade.trainer.engine import VectorEngine  # noqa: E402

E = 64
cfg = _cfg(False)
cfg.agent.target_every = 5
prices = _prices(E, seed=21)
dev = torch.device("cuda", 0)
eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
L = eng.layout
sig = [(5 * u + 3) % 128 for u in range(128)]
inv = [0] * 128
for u, v in enumerate(sig):
    inv[v] = u
bad = []
for mode in ("perm", "bias", "b2"):
    for v in range(128 if mode != "b2" else 3):
        pt = torch.zeros_like(eng.params_target)
        if mode == "perm":
            for u in range(128):
                L.w(pt, 0)[u, 203] = (u + 1) / 128.0
                L.w(pt, 1)[sig[u], u] = 1.0
            L.w(pt, 2)[0, v] = 1.0
            want = (inv[v] + 1) / 128.0
        elif mode == "bias":
            L.b(pt, 1)[v] = (v + 1) / 128.0
            L.w(pt, 2)[1, v] = 1.0
            want = (v + 1) / 128.0
        else:
            L.b(pt, 2)[v] = 0.25 * (v + 1)
            want = 0.25 * (v + 1)
        eng.params_target.copy_(pt)
        native.check(native.lib().st_qtarget_launch(eng._qtp, eng._qt_grid, native.stream_handle()), "qt")
        torch.cuda.synchronize()
        qt = eng.qt_buf.view(E, 3, 4).cpu()
        row = {"perm": 0, "bias": 1, "b2": v}[mode]
        got = qt[:, :, row]
        if float((got - want).abs().max()) > 1e-6:
            bad.append((mode, v, want, sorted(set(round(float(x), 6) for x in got.flatten().tolist()))[:4]))
        others = [r for r in range(3) if r != row]
        if float(qt[:, :, others].abs().max()) > 1e-6 and mode != "b2":
            bad.append((mode, v, "other rows nonzero", float(qt[:, :, others].abs().max())))
for b in bad[:60]:
    print(b)
print("bad:", len(bad))
