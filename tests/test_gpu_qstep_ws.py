"""Numerics of the wave-specialised fused step kernel (csrc/qstep_ws.hip) vs the plain-PyTorch fp32 oracle
and vs the 64-env-chunk kernel (csrc/qstep_wide.hip).

The oracle (`sharetrade.env.trading.engine_step_ref`) rounds to bf16 at the same points as the kernel
(``emulate_bf16=True``).  Actions agree except on near-ties of Q (the fp32 summation order inside the
MFMAs differs); with the kernel's actions forced into the oracle, env transitions and rewards must match
exactly and the gradient within a relative-norm tolerance.  Small ``engine.grid`` values make every
workgroup run many tiles, so the LDS ring of the kernel wraps around many times.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


# csrc/qstep_ws.hip; the retired csrc/ab/qstep_pipe.hip (same contract, same checks) only with SHARETRADE_AB_BUILDS=1
KERNELS = ["ws"] + (["pipe"] if os.environ.get("SHARETRADE_AB_BUILDS", "") not in ("", "0") else [])


def _cfg(compat=False, kernel="ws"):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship")
    cfg.engine.step_kernel = kernel
    # a tuning build of the ws kernel (csrc/qstep_ws_<v>.hip) under the same checks, for A/B candidates
    cfg.engine.step_variant = os.environ.get("SHARETRADE_WS_VARIANT", "") if kernel == "ws" else ""
    if compat:
        cfg.env.compat_decisions = True
        cfg.agent.target_slot = "compat"
        cfg.model.output_relu = True
    return cfg


def _prices(E, T=400, seed=3, tick16=True):
    """Random-walk banks on the 16-bit tick grid (data.tick16, as the engine's synthetic banks): the ws kernel then
    reads its windows as u16 ticks (the production path); ``tick16=False`` keeps arbitrary fp32 prices (its fp32
    window path)."""
    from sharetrade.data.prices import random_walk, tick16_quantize

    p = random_walk(T, 50.0, 0.02, seed, n_series=E).astype(np.float32)
    return torch.from_numpy(tick16_quantize(p) if tick16 else p)


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def _oracle(cfg, prices, st0, params, layout, step, loss_coef, **kw):
    from sharetrade.env import trading as tr

    return tr.engine_step_ref(
        prices, st0.to("cpu"), params, layout, history=cfg.model.history, feature_mode=cfg.env.features,
        budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
        target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
        epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=step,
        loss_coef=loss_coef, reward_mode=cfg.agent.reward_mode, td_clip=cfg.agent.td_clip, **kw)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("compat", [False, True])
@pytest.mark.parametrize("E,grid", [(64, 0), (256, 0), (640, 2), (1024, 3), (4096, 0)])
def test_ws_matches_oracle(native_built, kernel, compat, E, grid):
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg(compat, kernel)
    cfg.agent.epsilon = 0.5
    cfg.engine.grid = grid
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    assert eng.step_kernel == kernel
    st0 = eng.state.clone()
    st0.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 3 % 190)
    st0.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 3)
    st0.value.copy_(prices[:, 0].to(dev))
    for k in st0.as_dict():
        getattr(eng.state, k).copy_(getattr(st0, k))
    eng.ctrl.fill_(5)
    params = eng.params.detach().cpu().clone()
    grad = eng.native_grad().detach().cpu().clone()
    torch.cuda.synchronize()
    assert int(eng.kernel_err.sum()) == 0, "ring wait gave up"
    acts = eng.actions_out.cpu().clone()
    rew = eng.rewards_out.cpu().clone()
    _, _, info0 = _oracle(cfg, prices, st0, params, eng.layout, 5, eng.loss_coef, emulate_bf16=True)
    mism = (info0["actions"].cpu() != acts).float().mean().item()
    print(f"[meas] oracle {kernel} compat={compat} E={E} grid={grid} action_mismatch={mism:.4f}")
    # bounds ~2x the largest measured value over these cases (profiles/r5_ws_numerics.md): relative errors
    # <= 1.7e-3 vs the bf16-emulating oracle, <= 1.65e-2 vs pure fp32; actions: 0 mismatches measured, 1 %
    # left for near-ties of Q (the fp32 summation order inside the MFMAs differs)
    assert mism <= 0.01, f"action mismatch rate {mism}"
    ns, g_ref, info = _oracle(cfg, prices, st0, params, eng.layout, 5, eng.loss_coef, emulate_bf16=True,
                              forced_actions=acts)
    assert torch.equal(info["reward"], rew)
    for k in ("budget", "shares", "value", "pos", "episodes"):
        assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), k
    L = eng.layout
    for l in range(L.n_layers):
        gw, rw = L.w(grad, l), L.w(g_ref, l)
        print(f"[meas] oracle {kernel} compat={compat} E={E} layer={l} w_rel_bf16={_rel(gw, rw):.3e}"
              + (f" b_rel_bf16={_rel(L.b(grad, l), L.b(g_ref, l)):.3e}" if l > 0 else ""))
        assert _rel(gw, rw) < 5e-3, (l, _rel(gw, rw))
        if l > 0:
            assert _rel(L.b(grad, l), L.b(g_ref, l)) < 5e-3, l
    # and vs the pure fp32 oracle (no bf16 emulation, same actions): the bound the wide kernel meets
    _, g32, _ = _oracle(cfg, prices, st0, params, eng.layout, 5, eng.loss_coef, emulate_bf16=False,
                        forced_actions=acts)
    print(f"[meas] oracle {kernel} compat={compat} E={E} grad_rel_fp32={_rel(grad, g32):.3e}")
    assert _rel(grad, g32) < 3.5e-2, _rel(grad, g32)
    # statistics slab: reward sum and the number of explore draws
    st = eng.stat_slab.sum(0).cpu()
    assert abs(float(st[0]) - float(info["reward"].sum())) < 1e-3 + 1e-4 * float(info["reward"].abs().sum())
    assert int(round(float(st[2]))) == int((~info0["exploit"]).sum())


@pytest.mark.parametrize("kernel", KERNELS)
def test_ws_episode_end_and_reset(native_built, kernel):
    """Envs at the last position of their series finish the episode in this step: last_final, episode
    counter and the reset of budget / shares / position written by the data waves."""
    from sharetrade.trainer.engine import VectorEngine

    E, T = 256, 260
    cfg = _cfg(kernel=kernel)
    prices = _prices(E, T=T, seed=9)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    st0 = eng.state.clone()
    st0.pos.copy_(torch.full((E,), T - 201 - 1, dtype=torch.int32, device=dev))
    st0.pos[::2] = 10
    st0.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 2)
    st0.value.copy_(prices[:, 5].to(dev))
    for k in st0.as_dict():
        getattr(eng.state, k).copy_(getattr(st0, k))
    eng.ctrl.fill_(3)
    params = eng.params.detach().cpu().clone()
    eng.native_grad()
    torch.cuda.synchronize()
    acts = eng.actions_out.cpu().clone()
    ns, _, _ = _oracle(cfg, prices, st0, params, eng.layout, 3, eng.loss_coef, emulate_bf16=True,
                       forced_actions=acts)
    for k in ("budget", "shares", "value", "pos", "episodes", "ret_sum"):
        assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), k
    done = ns.episodes.cpu() > 0
    assert int(done.sum()) == E // 2
    assert torch.equal(ns.last_final[done], eng.state.last_final.cpu()[done])


def test_ws_and_wide_agree_over_steps(native_built):
    """Ten captured steps of each kernel from the same start: the learned parameters stay close (both are
    bf16 MFMA steps of the same math; fp32 summation orders differ) and the env statistics agree."""
    from sharetrade.trainer.engine import VectorEngine

    E = 2048
    prices = _prices(E, seed=4)
    dev = torch.device("cuda", 0)
    out = {}
    for kern in ["wide"] + KERNELS:
        cfg = _cfg(kernel=kern)
        cfg.agent.epsilon = 0.0          # every action a uniform draw: identical trajectories
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.step_kernel == kern
        eng.capture_graph(warmup=1)
        eng.run(10)
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        out[kern] = (eng.params.detach().cpu().clone(), {k: v.cpu().clone() for k, v in eng.state.as_dict().items()},
                     eng.stat_acc.cpu().clone())
    pw, sw, stw = out["wide"]
    for kern in KERNELS:
        pv, sv, stv = out[kern]
        for k in ("budget", "shares", "pos", "value"):
            assert torch.equal(sw[k], sv[k]), (kern, k)
        print(f"[agree] {kern} vs wide: params rel {_rel(pv, pw):.3e}")
        assert _rel(pv, pw) < 1e-2, (kern, _rel(pv, pw))
        assert torch.allclose(stv[0], stw[0], rtol=1e-5, atol=1e-5), kern     # reward sums
        assert torch.allclose(stv[1], stw[1], rtol=2e-2), kern                # TD loss sums


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("compat", [False, True])
def test_ws_trajectory_matches_torch_oracle(native_built, kernel, compat):
    """Ten eager ws steps against the plain-PyTorch oracle engine (engine_step_ref + optimizer_step_ref)
    driven with the kernel's actions: env transitions and rewards exact at every step, the learned
    parameter change within bf16 tolerance of the oracle's (bf16-emulating forward / backward) and
    within a looser bound of the pure-fp32 oracle's.  SGD, so the parameter change is linear in the
    gradients (Adam's first steps are ~lr * sign(g): elements with near-zero gradients would flip)."""
    from sharetrade.models import qnet as qn
    from sharetrade.trainer.engine import VectorEngine

    E = 1024
    cfg = _cfg(compat, kernel)
    cfg.agent.epsilon = 0.6
    cfg.agent.optimizer = "sgd"
    cfg.agent.lr = 0.01
    prices = _prices(E, T=320, seed=11)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    assert eng.step_kernel == kernel
    eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 5 % 100)
    refs = {}
    for emulate in (True, False):
        ref = VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")
        ref.params.copy_(eng.params.detach().cpu())
        refs[emulate] = ref
    p0 = eng.params.detach().cpu().clone()
    a = cfg.agent
    for t in range(10):
        st0 = eng.state.clone().to("cpu")
        eng.step()
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        acts = eng.actions_out.cpu().clone()
        rew = eng.rewards_out.cpu().clone()
        for emulate, ref in refs.items():
            ns, g, info = _oracle(cfg, prices, st0, ref.params, ref.layout, t, eng.loss_coef,
                                  emulate_bf16=emulate, forced_actions=acts)
            qn.optimizer_step_ref(ref.params, g, ref.opt, ref.mask, a.lr, a.adam_betas, a.adam_eps)
            if emulate:
                assert torch.equal(info["reward"], rew), t
                for k in ("budget", "shares", "value", "pos", "episodes"):
                    assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), (t, k)
    d = eng.params.detach().cpu() - p0
    for emulate, tol in ((True, 5e-4), (False, 5e-3)):   # measured 2.0e-4 / 2.2e-3
        dr = refs[emulate].params - p0
        print(f"[meas] trajectory {kernel} compat={compat} emulate_bf16={emulate} dparam_rel={_rel(d, dr):.3e}")
        assert _rel(d, dr) < tol, (emulate, _rel(d, dr))


@pytest.mark.parametrize("kernel", KERNELS)
def test_ws_adam_trajectory_matches_torch_oracle(native_built, kernel):
    """Three eager steps with the flagship's Adam against the oracle engine driven with the kernel's actions.
    Adam's first steps move each parameter by ~lr * sign(m): elements whose accumulated gradient is near zero
    can flip, so the check is on the optimizer moments (linear / quadratic in the gradients) and on the
    parameter change of the elements with a clear gradient (|m| above its median)."""
    from sharetrade.models import qnet as qn
    from sharetrade.trainer.engine import VectorEngine

    E = 2048
    cfg = _cfg(False, kernel)
    cfg.agent.epsilon = 0.6
    assert cfg.agent.optimizer == "adam"
    prices = _prices(E, T=320, seed=23)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 5 % 100)
    ref = VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")
    ref.params.copy_(eng.params.detach().cpu())
    p0 = eng.params.detach().cpu().clone()
    a = cfg.agent
    for t in range(3):
        st0 = eng.state.clone().to("cpu")
        eng.step()
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        acts = eng.actions_out.cpu().clone()
        ns, g, info = _oracle(cfg, prices, st0, ref.params, ref.layout, t, eng.loss_coef, emulate_bf16=True,
                              forced_actions=acts)
        qn.optimizer_step_ref(ref.params, g, ref.opt, ref.mask, a.lr, a.adam_betas, a.adam_eps)
        assert torch.equal(info["reward"], eng.rewards_out.cpu()), t
        for k in ("budget", "shares", "value", "pos"):
            assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), (t, k)
    m, v = eng.opt.s1.cpu(), eng.opt.s2.cpu()
    mr, vr = ref.opt.s1, ref.opt.s2
    clear = mr.abs() > mr.abs()[ref.mask.bool()].median()
    d, dr = (eng.params.detach().cpu() - p0)[clear], (ref.params - p0)[clear]
    print(f"[meas] adam trajectory {kernel} m_rel={_rel(m, mr):.3e} v_rel={_rel(v, vr):.3e} "
          f"dparam_rel(clear)={_rel(d, dr):.3e} sign_flips={(torch.sign(d) != torch.sign(dr)).float().mean():.4f}")
    # measured 3.1e-4 / 3.1e-4 / 1.7e-4, no sign flips (profiles/r5_ws_numerics.md)
    assert _rel(m, mr) < 7e-4 and _rel(v, vr) < 7e-4, (_rel(m, mr), _rel(v, vr))
    assert _rel(d, dr) < 4e-4, _rel(d, dr)


def test_tick16_kernel_matches_host_mirror(native_built):
    """csrc/series.hip tick16 (mode 0: quantize in place) equals data.prices.tick16_quantize bit for bit; its
    ticks times the row scale give the quantized prices back; mode 1 accepts a bank on the grid and rejects one
    off it; the engine's synthetic random-walk bank is on the grid."""
    from sharetrade.data.prices import random_walk, tick16_quantize
    from sharetrade.ops import native
    from sharetrade.trainer.engine import make_price_bank

    p = random_walk(517, 50.0, 0.03, 3, n_series=300).astype(np.float32)
    p[7] *= 1e-3
    p[8] *= 1e5
    dev = torch.device("cuda", 0)
    g = torch.from_numpy(p).to(dev)
    assert native.tick16(g.clone(), quantize=False) is None              # off the grid
    native.tick16_quantize_(g)
    q = tick16_quantize(p)
    assert torch.equal(g.cpu(), torch.from_numpy(q))
    ticks, scale = native.tick16(g, quantize=False)                       # on the grid now
    t = ticks.cpu().numpy().view(np.uint16).astype(np.float32)
    assert np.array_equal(t[:, :517] * scale.cpu().numpy()[:, None], q)
    assert not t[:, 517:].any()
    cfg = _cfg()
    cfg.data.length = 700
    bank = make_price_bank(cfg, 128, dev, seed=1)
    assert native.tick16(bank, quantize=False) is not None


@pytest.mark.parametrize("knobs", [False, True])
def test_ws_tick_bank_bit_identical_to_fp32_windows(native_built, knobs):
    """The 16-bit tick windows (engine.bank16='auto' on a bank on the tick grid) against the fp32 windows of the
    same bank (bank16='off'): features are the same numbers (w / last - 1 = tick_w / tick_last - 1 exactly), so
    6 captured steps give bit-identical parameters, optimizer state, env state and statistics -- with the
    learning knobs, the target pass (csrc/qtarget.hip) on ticks too.  Positions spread so both odd and even
    window starts occur in every tile.  And a bank off the grid keeps the fp32 path."""
    from sharetrade.trainer.engine import VectorEngine

    E = 2048
    prices = _prices(E, T=330, seed=31)
    dev = torch.device("cuda", 0)
    out = {}
    for b16 in ("auto", "off"):
        cfg = _cfg()
        cfg.engine.bank16 = b16
        cfg.agent.epsilon = 0.7
        if knobs:
            cfg.agent.target_every, cfg.agent.double_dqn, cfg.agent.reward_scale = 2, True, 3.0
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert (eng.ticks is not None) == (b16 == "auto")
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 13 % 120)
        eng.capture_graph(warmup=1)
        eng.run(6)
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        out[b16] = [eng.params.detach().cpu().clone(), eng.opt.s1.cpu().clone(), eng.opt.s2.cpu().clone(),
                    eng.stat_acc.cpu().clone()] + [v.cpu().clone() for v in eng.state.as_dict().values()]
    for x, y in zip(out["auto"], out["off"]):
        if x.is_floating_point():
            x, y = x.view(torch.int32) if x.dtype == torch.float32 else x.view(torch.int64), \
                   y.view(torch.int32) if y.dtype == torch.float32 else y.view(torch.int64)
        assert torch.equal(x, y)
    cfg = _cfg()
    eng = VectorEngine(cfg, prices=_prices(256, T=330, seed=31, tick16=False), device=dev, envs=256)
    assert eng.ticks is None and eng.prices4 is not None


def test_ws_weight_image_stays_equal_to_fresh_pack(native_built, monkeypatch):
    """The ws prologue DMA-copies a weight image that the optimizer keeps current by scatter writes (img_map).
    After several Adam steps it equals a fresh pack of the parameters byte for byte, and a run with the image
    (SHARETRADE_WS_WIMG=1, the default) is bit-identical to one that gathers the images from wq / wf (=0) in
    parameters, optimizer moments and env state (a stale map entry would otherwise hide inside the
    trajectory tolerances)."""
    from sharetrade.ops import native
    from sharetrade.trainer.engine import VectorEngine

    E = 1024
    prices = _prices(E, T=320, seed=29)
    dev = torch.device("cuda", 0)
    out = {}
    for wimg in ("1", "0"):
        monkeypatch.setenv("SHARETRADE_WS_WIMG", wimg)
        cfg = _cfg()
        cfg.agent.epsilon = 0.6
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert (eng._wimg is not None) == (wimg == "1")
        eng.run(5)
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        if wimg == "1":
            fresh, _ = native.ws_weight_image(eng.params, eng.layout.segments)
            assert torch.equal(eng._wimg, fresh)
        out[wimg] = (eng.params.detach().cpu().clone(), eng.opt.s1.cpu().clone(), eng.opt.s2.cpu().clone(),
                     {k: v.cpu().clone() for k, v in eng.state.as_dict().items()})
    a, b = out["1"], out["0"]
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    for k in a[3]:   # (bit patterns: last_final holds NaN until an episode completes)
        x, y = a[3][k], b[3][k]
        if x.is_floating_point():
            x, y = x.view(torch.int32), y.view(torch.int32)
        assert torch.equal(x, y), k


@pytest.mark.parametrize("E,grid", [(64 * 48, 16), (64 * 100, 8), (64 * 13, 8), (64 * 1000, 16), (64 * 2048, 256)])
def test_ws_dynamic_schedule_matches_static(native_built, E, grid):
    """csrc/qstep_ws.hip with the dynamic chunk schedule (overlapped DP): rounds 0-2 static, later chunks
    claimed from per-XCD-group heads and handed to the data waves through the LDS ring, the gradient
    waves stopping at the round count.  Every chunk is stepped exactly once per launch, transitions and
    actions equal the static schedule's, gradients agree up to the bf16 rounding of differently grouped
    partials; the heads are re-zeroed so a second launch works too."""
    from sharetrade.trainer.engine import VectorEngine

    prices = _prices(E, seed=5)
    dev = torch.device("cuda", 0)
    out = {}
    for sched in ("static", "dynamic"):
        cfg = _cfg()
        cfg.agent.epsilon = 0.5
        cfg.engine.chunk_schedule = sched
        cfg.engine.grid = grid
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.step_kernel == "ws" and eng.chunk_schedule == sched and eng.grid == grid
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 5 % 150)
        pos0 = eng.state.pos.clone()
        eng.ctrl.fill_(7)
        g = eng.native_grad().detach().cpu().clone()
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0, "ring wait gave up"
        assert torch.equal(eng.state.pos, pos0 + 1), "a chunk was skipped or stepped twice"
        out[sched] = (g, eng.actions_out.cpu().clone(), eng.stat_slab.sum(0).cpu(),
                      {k: v.cpu().clone() for k, v in eng.state.as_dict().items()})
        if sched == "dynamic":
            assert int(eng.chunk_heads.abs().sum()) == 0, "claim heads not re-zeroed"
            g2 = eng.native_grad().detach().cpu().clone()
            torch.cuda.synchronize()
            assert int(eng.kernel_err.sum()) == 0
            assert torch.equal(eng.state.pos, pos0 + 2)
            assert torch.isfinite(g2).all()
    gs, as_, sts, ss = out["static"]
    gd, ad, std_, sd = out["dynamic"]
    assert torch.equal(ad, as_)
    for k in ("budget", "shares", "value", "episodes"):
        assert torch.equal(ss[k], sd[k]), k
    assert _rel(gd, gs) < 4e-3, _rel(gd, gs)
    assert torch.allclose(std_, sts, rtol=1e-4, atol=1e-3)


def test_ws_dynamic_schedule_multi_step_graphs(native_built):
    """The dynamic-schedule ws kernel inside captured multi-step graphs (the heads are re-zeroed between
    launches by the slab pass): the same trajectory as the static schedule over 12 steps."""
    from sharetrade.trainer.engine import VectorEngine

    E = 64 * 512
    prices = _prices(E, seed=6)
    dev = torch.device("cuda", 0)
    res = {}
    for sched in ("static", "dynamic"):
        cfg = _cfg()
        cfg.agent.epsilon = 0.0   # uniform actions: identical trajectories
        cfg.engine.chunk_schedule = sched
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.chunk_schedule == sched
        eng.capture_graph(warmup=1, graph_steps=4)
        eng.run(12)
        torch.cuda.synchronize()
        assert int(eng.kernel_err.sum()) == 0
        res[sched] = (eng.params.cpu().clone(), {k: v.cpu().clone() for k, v in eng.state.as_dict().items()})
    (ps, ss), (pd, sd) = res["static"], res["dynamic"]
    for k in ("budget", "shares", "pos", "value"):
        assert torch.equal(ss[k], sd[k]), k
    assert _rel(pd, ps) < 1e-2, _rel(pd, ps)
