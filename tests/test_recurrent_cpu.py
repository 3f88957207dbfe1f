"""Config 5 (GRU recurrent Q-net) host pieces: MX-fp8 reference quantizer, minute-bar
generator, torch GRU reference and the minute-bar env semantics (CPU only)."""
import numpy as np
import torch

from sharetrade.data import minute_bars as mb
from sharetrade.env import minute as me
from sharetrade.models import gru_qnet as gq
from sharetrade.ops.gru import mx_exp, mx_quantize, mx_roundtrip


def test_mx_exponent_rule():
    a = torch.tensor([1.0, 448.0, 448.5, 896.0, 1e-3, 3.0e-38, 0.0])
    e = mx_exp(a)
    for v, k in zip(a.tolist(), e.tolist()):
        if v == 0:
            assert k == -127
            continue
        assert v / 2.0 ** k <= 448.0                          # never saturates
        if k > -127:
            assert v / 2.0 ** (k - 1) > 448.0                 # smallest such exponent
    assert e.tolist()[:4] == [-8, 0, 1, 1]


def test_mx_roundtrip_error_bound():
    x = torch.randn(64, 256) * torch.logspace(-3, 2, 64)[:, None]
    y = mx_roundtrip(x)
    q, e = mx_quantize(x)
    assert q.dtype == torch.float8_e4m3fn and e.shape == (64, 8)
    blk = x.view(64, 8, 32).abs().amax(-1, keepdim=True)
    err = (y - x).view(64, 8, 32).abs()
    # e4m3: 3 mantissa bits -> half-ulp <= 2^-4 relative of the element; plus subnormal floor
    assert bool((err <= x.view(64, 8, 32).abs() * 2 ** -4 + blk * 2 ** -9 + 1e-30).all())


def test_minute_bars_numpy_is_deterministic_and_sane():
    c1, f1 = mb.generate_numpy(16, 500, seed=1)
    c2, f2 = mb.generate_numpy(16, 500, seed=1)
    c3, _ = mb.generate_numpy(16, 500, seed=2)
    assert np.array_equal(c1, c2) and np.array_equal(f1, f2) and not np.array_equal(c1, c3)
    assert c1.shape == (16, 500) and f1.shape == (16, 500, 8)
    assert np.isfinite(f1).all() and (c1 > 0).all()
    r = np.diff(np.log(c1), axis=1)
    assert 0.0 < np.mean(r[:, 1:] * r[:, :-1]) / np.mean(r * r) < 0.3      # AR(1) momentum edge
    assert np.allclose(f1[:, 1:, 0], r * 100, rtol=1e-3, atol=1e-3)


def test_gru_reference_matches_torch_grucell():
    p = gq.init_params(seed=3)
    cell = torch.nn.GRUCell(64, 256)
    with torch.no_grad():
        cell.weight_ih.copy_(p["w_ih"]); cell.weight_hh.copy_(p["w_hh"])
        cell.bias_ih.copy_(p["b_ih"]); cell.bias_hh.copy_(p["b_hh"])
    x, h = torch.randn(7, 64), torch.randn(7, 256)
    assert torch.allclose(cell(x, h), gq.gru_cell(x, h, p), atol=1e-6)


def test_sequence_loss_masks_and_backprops():
    p = {k: v.clone().requires_grad_(True) for k, v in gq.init_params(seed=4).items()}
    pt = {k: v.detach().clone() for k, v in p.items()}
    S, B = 6, 5
    X = torch.randn(S + 1, B, 64)
    X[..., 32:] = 0
    A = torch.randint(0, 3, (S, B))
    R = torch.randn(S, B)
    D = torch.zeros(S, B)
    D[2, 1] = 1
    loss = gq.sequence_td_loss(p, pt, X, torch.zeros(B, 256), A, R, D, 0.99, burn=2)
    loss.backward()
    assert torch.isfinite(loss) and all(torch.isfinite(t.grad).all() for t in p.values())
    assert float(p["w_ih"].grad[:, 32:].abs().max()) == 0.0     # padded x columns get no gradient
    # a reset cuts the recurrence: h after the done step restarts from zero
    q1, _ = gq.unroll(X, torch.zeros(B, 256), pt, D)
    X2 = X.clone()
    X2[:3, 1] += 5.0                                           # perturb env 1 before its reset
    q2, _ = gq.unroll(X2, torch.zeros(B, 256), pt, D)
    assert torch.allclose(q1[3:, 1], q2[3:, 1]) and not torch.allclose(q1[:3, 1], q2[:3, 1])


def test_minute_env_semantics():
    close = np.array([10.0, 11.0, 12.1, 12.1, 13.0, 14.0, 15.0, 16.0, 17.0, 18.0], np.float32)
    ret = mb.bar_returns(close[None])[0]
    assert abs(ret[0] - 10.0) < 1e-4 and ret[-1] == 0
    st = me.MinuteEnvState(t=0, es=0)
    r, done, _ = me.step(st, 0, close, ret, len(close), 3, 0.5, 0.0)         # buy at 10 -> +10% - cost
    assert st.pz == 1 and st.entry == 10.0 and not done
    assert abs(r - (10.0 - 0.5)) < 1e-4
    r, done, _ = me.step(st, 2, close, ret, len(close), 3, 0.5, 0.0)         # hold long 11 -> 12.1
    assert abs(r - 10.0) < 1e-3 and st.pz == 1
    x = me.obs(np.zeros(8, np.float32), close[st.t], st, 3)
    assert x[8] == 1 and abs(x[9] - 21.0) < 1e-3 and abs(x[10] - 2 / 3) < 1e-6 and x[11] == 1
    r, done, fin = me.step(st, 1, close, ret, len(close), 3, 0.5, 0.5)       # sell (flat: 0 - cost), episode ends
    assert done and abs(r + 0.5) < 1e-6 and st.pz == 0 and st.episodes == 1
    assert abs(fin - (9.5 + 10.0 - 0.5)) < 1e-3
    assert st.es == min(int(np.float32(0.5) * np.float32(len(close) - 3 - 1)), len(close) - 3 - 2) == st.t
    r, _, _ = me.step(st, 1, close, ret, len(close), 3, 0.5, 0.0)            # sell while flat: no trade
    assert r == 0.0 and st.pz == 0
