"""CPU tests of the reference-semantics oracle (BASELINE.json config 1 plumbing)."""
import os

import numpy as np
import pytest
import torch

from sharetrade.config import default_csv_path, preset_config
from sharetrade.env import trading as tr
from sharetrade.models import qnet as qn
from sharetrade.utils import rng


def test_layout_padding_and_bias_fold():
    L = qn.QNetLayout(203, [200], 3)
    assert L.pdims == [224, 224, 16]
    assert L.bias_col == 203
    flat = torch.arange(L.numel, dtype=torch.float32)
    assert L.w(flat, 0).shape == (224, 224)
    assert L.b(flat, 0).shape == (224,)
    assert L.n_real_params() == 203 * 200 + 200 + 200 * 3 + 3
    L2 = qn.QNetLayout(203, [128, 128], 3)
    assert L2.pdims == [224, 128, 128, 16]
    for s in L2.segments.values():
        assert s.offset % qn.SEG_ALIGN == 0


def test_forward_matches_plain_mlp():
    m = preset_config("reference_compat").model
    L = qn.QNetLayout.from_config(m)
    p = qn.init_params(L, m, seed=3)
    x = torch.randn(5, 203)
    q, _, _ = qn.forward(p, L, x, output_relu=True)
    W1 = L.w(p, 0)[:200, :203]
    b1 = L.b(p, 0)[:200]
    W2 = L.w(p, 1)[:3, :200]
    b2 = L.b(p, 1)[:3]
    ref = torch.relu(torch.relu(x @ W1.t() + b1) @ W2.t() + b2)
    assert torch.allclose(q[:, :3], ref, rtol=1e-4, atol=1e-3)
    assert torch.all(q[:, 3:] == 0)
    # reference init: biases 0.1 (tf.constant), weights ~N(0,1)
    assert torch.all(b1 == 0.1) and torch.all(b2 == 0.1)
    assert abs(float(W1.std()) - 1.0) < 0.05


def test_backward_matches_autograd():
    m = preset_config("flagship").model
    L = qn.QNetLayout.from_config(m)
    p = qn.init_params(L, m, seed=1)
    x = torch.randn(7, 203)
    q, acts, xp = qn.forward(p, L, x, output_relu=False)
    dq = torch.zeros_like(q)
    dq[:, :3] = torch.randn(7, 3)
    g = qn.backward(p, L, xp, acts, q, dq, output_relu=False)
    pa = p.clone().requires_grad_(True)
    qa, _, _ = qn.forward(pa, L, x, output_relu=False)
    (qa * dq).sum().backward()
    assert torch.allclose(g, pa.grad, rtol=1e-4, atol=1e-4)


def test_philox_known_answer_and_vectorised():
    # Random123 known-answer vector for philox4x32-10 with zero counter / key
    r = rng.philox4x32(np.uint32(0), np.uint32(0), np.uint32(0), np.uint32(0), np.uint32(0), np.uint32(0))
    assert [int(v) for v in r] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    u1, u2 = rng.uniforms(5, 0, np.arange(100), 17)
    u1b, _ = rng.uniforms(5, 0, np.arange(100), 17)
    assert np.array_equal(u1, u1b)
    assert (u1 >= 0).all() and (u1 < 1).all()
    assert not np.array_equal(u1, rng.uniforms(5, 1, np.arange(100), 17)[0])


def test_env_transition_rules():
    b = torch.tensor([100.0, 100.0, 5.0, 100.0])
    s = torch.tensor([0, 2, 0, 1], dtype=torch.int32)
    a = torch.tensor([0, 1, 0, 2], dtype=torch.int32)   # Buy, Sell, Buy(unaffordable), Hold
    v_prev = torch.tensor([10.0, 10.0, 10.0, 10.0])
    v_new = torch.tensor([10.0, 12.0, 10.0, 11.0])
    b2, s2, r = tr.env_transition(a, b, s, v_prev, v_new, compat=False, b0=2400.0, s0=0)
    assert b2.tolist() == [90.0, 112.0, 5.0, 100.0]
    assert s2.tolist() == [1, 1, 0, 1]
    assert r.tolist() == pytest.approx([0.0, 4.0, 0.0, 1.0])


def test_compat_msft_run_reproduces_reference_portfolio():
    """Reference quirk Q1: every worker ends at exactly its initial budget."""
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("reference_compat")
    cfg.engine.envs_per_rank = 2
    eng = VectorEngine(cfg, device=torch.device("cpu"))
    assert eng.T == 6047
    eng.run(30)
    s = eng.stats_dict()
    assert s["reward_sum"] == 0.0
    assert torch.all(eng.current_portfolios() == 2400.0)


def test_ar1_price_bank_has_momentum():
    """data.source = "ar1": log-returns with lag-1 autocorrelation ~phi (the learnable signal of
    tools/learning_curve.py); prices positive, first column the start price."""
    import torch

    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import make_price_bank

    cfg = preset_config("flagship")
    cfg.data.source, cfg.data.ar_phi, cfg.data.length = "ar1", 0.3, 2000
    bank = make_price_bank(cfg, 128, torch.device("cpu"))
    assert bank.shape == (128, 2000) and bool((bank > 0).all())
    assert torch.allclose(bank[:, 0], torch.full((128,), cfg.data.start_price))
    r = torch.log(bank[:, 1:].double() / bank[:, :-1].double())
    a, b = r[:, 1:] - r[:, 1:].mean(), r[:, :-1] - r[:, :-1].mean()
    rho = float((a * b).sum() / (a.norm() * b.norm()))
    assert abs(rho - 0.3) < 0.03, rho


def test_philox_init_is_normal_and_counter_based():
    """model.init_rng = "philox": W ~ N(0, std) from the counter-based generator (host mirror of
    csrc/series.hip init_normal_kernel); padding stays zero; the values depend only on (seed, layer,
    index), not on the padded layout."""
    from sharetrade.models import qnet as qn

    cfg = preset_config("reference_compat")
    L = qn.QNetLayout.from_config(cfg.model)
    p = qn.init_params(L, cfg.model, seed=11)
    w0 = L.w(p, 0)
    real = w0[: L.dims[1], : L.dims[0]]
    assert abs(float(real.mean())) < 0.01 and abs(float(real.std()) - 1.0) < 0.01
    assert float(w0[L.dims[1]:].abs().sum()) == 0.0 and float(w0[:, L.dims[0] + 1:].abs().sum()) == 0.0
    assert torch.equal(real, qn.philox_normal(L.dims[1], L.dims[0], 1.0, 11, 0))
    assert not torch.equal(p, qn.init_params(L, cfg.model, seed=12))
    assert torch.equal(p, qn.init_params(L, cfg.model, seed=11))
