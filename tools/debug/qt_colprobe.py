"""Column probe of csrc/qtarget.hip: a target net that passes input column c straight to Q[0]
(W0 rows 0 / 1 = +e_c / -e_c, W1 rows 0 / 1 = e_0 / e_1, W2 row 0 = (1, -1)), so QT[e][a][0] = x'_a[e][c]."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from test_gpu_qstep_ws import _cfg, _oracle, _prices  # noqa: E402

from sharetrade.ops import native  # noqa: E402
from sharetrade.trainer.engine import VectorEngine  # noqa: E402

E = 64
cfg = _cfg(False)
cfg.agent.target_every = 5
prices = _prices(E, seed=21)
dev = torch.device("cuda", 0)
eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 7 % 190)
eng.state.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 4)
eng.state.budget.copy_(torch.linspace(0.0, 3.0 * cfg.env.budget, E, device=dev))
st0 = eng.state.clone().to("cpu")
L = eng.layout
xs = []
for act in range(3):
    _, _, info = _oracle(cfg, prices, st0, eng.params.detach().cpu(), L, 0, eng.loss_coef, emulate_bf16=True,
                         forced_actions=torch.full((E,), act, dtype=torch.int32))
    xs.append(info["x_next"].to(torch.bfloat16).float())
bad = []
for c, k in [(c, c % 64) for c in range(204)] + [(c, (7 * c + 3) % 64) for c in range(204)]:
    pt = torch.zeros_like(eng.params_target)
    L.w(pt, 0)[2 * k, c] = 1.0
    L.w(pt, 0)[2 * k + 1, c] = -1.0
    L.w(pt, 1)[2 * k, 2 * k] = 1.0
    L.w(pt, 1)[2 * k + 1, 2 * k + 1] = 1.0
    L.w(pt, 2)[0, 2 * k] = 1.0
    L.w(pt, 2)[0, 2 * k + 1] = -1.0
    eng.params_target.copy_(pt)
    native.check(native.lib().st_qtarget_launch(eng._qtp, eng._qt_grid, native.stream_handle()), "qt")
    torch.cuda.synchronize()
    qt = eng.qt_buf.view(E, 3, 4).cpu()
    for act in range(3):
        got = qt[:, act, 0]
        want = xs[act][:, c] if c < 203 else torch.ones(E)
        err = float((got - want).abs().max())
        if err > 1e-3:
            # which column of x' does it match?
            match = [cc for cc in range(203) if float((got - xs[act][:, cc]).abs().max()) < 1e-6]
            bad.append((c, k, act, err, match))
for b in bad[:60]:
    print("col %d pair %d act %d maxerr %.3e matches x' cols %s" % b)
print("bad entries:", len(bad))
