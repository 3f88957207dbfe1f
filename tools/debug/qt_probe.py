"""Where does csrc/qtarget.hip differ from the oracle's target forward?  Per action, per env group."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from test_gpu_qstep_ws import _cfg, _oracle, _prices, _rel  # noqa: E402

from sharetrade.models import qnet as qn  # noqa: E402
from sharetrade.trainer.engine import VectorEngine  # noqa: E402

E = 1024
cfg = _cfg(False)
cfg.agent.target_every = 5
prices = _prices(E, seed=21)
dev = torch.device("cuda", 0)
eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 7 % 190)
eng.state.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 4)
eng.state.budget.copy_(torch.linspace(0.0, 3.0 * cfg.env.budget, E, device=dev))
for perturb in (False, True):
    if perturb:
        g = torch.Generator().manual_seed(2)
        eng.params_target.add_((torch.randn(eng.params.shape, generator=g) * 0.02).to(dev) * eng._real)
    st0 = eng.state.clone().to("cpu")
    pt = eng.params_target.detach().cpu().clone()
    L = eng.layout
    import ctypes
    from sharetrade.ops import native
    native.check(native.lib().st_qtarget_launch(eng._qtp, eng._qt_grid, native.stream_handle()), "qt")
    torch.cuda.synchronize()
    qt = eng.qt_buf.view(E, 3, 4).cpu()
    for act in range(3):
        _, _, info = _oracle(cfg, prices, st0, eng.params.detach().cpu(), L, 0, eng.loss_coef, emulate_bf16=True,
                             forced_actions=torch.full((E,), act, dtype=torch.int32))
        ref, _, _ = qn.forward(pt, L, info["x_next"], cfg.model.output_relu, True)
        ref32, _, _ = qn.forward(pt, L, info["x_next"], cfg.model.output_relu, False)
        d = (qt[:, act, :3] - ref[:, :3]).abs().max(1).values
        print(f"perturb={perturb} act={act} rel={_rel(qt[:, act, :3], ref[:, :3]):.3e} "
              f"rel32={_rel(qt[:, act, :3], ref32[:, :3]):.3e} maxabs={float(d.max()):.3e} "
              f"frac>1e-2={float((d > 1e-2).float().mean()):.3f}")
        bad = torch.nonzero(d > 5 * d.median()).flatten()[:8].tolist()
        for e in bad:
            print(f"   env {e}: pos={int(st0.pos[e])} b={float(st0.budget[e]):.1f} s={int(st0.shares[e])} "
                  f"qt={qt[e, act, :3].tolist()} ref={ref[e, :3].tolist()}")
        print("   err by env%16:", [round(float(d[i::16].mean()), 5) for i in range(16)])
        print("   err by (env//16)%4:", [round(float(d.view(-1, 16)[j::4].mean()), 5) for j in range(4)])
