"""Numerics of the fused HIP engine step vs the plain-PyTorch fp32 oracle.

The oracle (`sharetrade.env.trading.engine_step_ref`) rounds to bf16 at the same
points as the kernel (``emulate_bf16=True``); accumulation order differs, so
gradients are compared with a relative-norm tolerance while env transitions
(fp32, no FMA contraction on either side) must match exactly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(compat=False):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship")
    if compat:
        cfg.env.compat_decisions = True
        cfg.agent.target_slot = "compat"
        cfg.model.output_relu = True
    return cfg


def _prices(E, T=400, seed=3):
    from sharetrade.data.prices import random_walk

    return torch.from_numpy(random_walk(T, 50.0, 0.02, seed, n_series=E).astype(np.float32))


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("compat", [False, True])
@pytest.mark.parametrize("E", [32, 96, 64, 192, 256])   # E % 64 == 0: csrc/qstep_wide.hip
def test_qstep_matches_oracle(native_built, compat, E):
    from sharetrade.env import trading as tr
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg(compat)
    cfg.agent.epsilon = 0.5
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    # advance positions so the epsilon ramp and shares are non-trivial
    st0 = eng.state.clone()
    st0.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 3 % 150)
    st0.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 3)
    st0.value.copy_(prices[:, 0].to(dev))
    for k in st0.as_dict():
        getattr(eng.state, k).copy_(getattr(st0, k))
    eng.ctrl.fill_(5)
    params = eng.params.detach().cpu().clone()
    grad = eng.native_grad().detach().cpu().clone()
    torch.cuda.synchronize()
    acts = eng.actions_out.cpu().clone()
    rew = eng.rewards_out.cpu().clone()

    # unforced oracle: the actions must agree except on near-ties of q
    ns_ref, g_ref0, info0 = tr.engine_step_ref(
        prices, st0.to("cpu"), params, eng.layout, history=cfg.model.history, feature_mode=cfg.env.features,
        budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
        target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
        epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=5,
        loss_coef=eng.loss_coef, reward_mode=cfg.agent.reward_mode, td_clip=cfg.agent.td_clip, emulate_bf16=True)
    mism = (info0["actions"].cpu() != acts).float().mean().item()
    assert mism <= 0.05, f"action mismatch rate {mism}"

    ns, g_ref, info = tr.engine_step_ref(
        prices, st0.to("cpu"), params, eng.layout, history=cfg.model.history, feature_mode=cfg.env.features,
        budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
        target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
        epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=5,
        loss_coef=eng.loss_coef, reward_mode=cfg.agent.reward_mode, td_clip=cfg.agent.td_clip, emulate_bf16=True, forced_actions=acts)
    assert torch.equal(info["reward"], rew)
    for k in ("budget", "shares", "value", "pos", "episodes"):
        assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), k
    # gradient vs oracle (bf16 activations, fp32 accumulation)
    L = eng.layout
    for l in range(L.n_layers):
        gw, rw = L.w(grad, l), L.w(g_ref, l)
        assert _rel(gw, rw) < 3e-2, (l, _rel(gw, rw))
        if l > 0:
            assert _rel(L.b(grad, l), L.b(g_ref, l)) < 3e-2
    # and vs the pure fp32 oracle (no bf16 emulation): looser
    _, g32, _ = tr.engine_step_ref(
        prices, st0.to("cpu"), params, eng.layout, history=cfg.model.history, feature_mode=cfg.env.features,
        budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
        target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
        epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=5,
        loss_coef=eng.loss_coef, reward_mode=cfg.agent.reward_mode, td_clip=cfg.agent.td_clip, emulate_bf16=False, forced_actions=acts)
    assert _rel(grad, g32) < 0.1


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("compat", [False, True])
def test_wide_and_narrow_kernels_agree(native_built, compat, waves):
    """csrc/qstep_wide.hip (64-env chunks) vs csrc/qstep_fused.hip (32-env chunks) on the same state:
    identical env transitions, gradients equal up to fp32 summation order."""
    from sharetrade.trainer.engine import VectorEngine

    E = 512
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    out = {}
    for chunk in (32, 64):
        cfg = _cfg(compat)
        cfg.agent.epsilon = 0.5
        cfg.engine.chunk = chunk
        cfg.engine.step_waves = waves
        cfg.engine.slab_dtype = "fp32"   # summation-order-only comparison (bf16 slabs: next test)
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.chunk == chunk
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 7 % 150)
        eng.ctrl.fill_(9)
        g = eng.native_grad().detach().cpu().clone()
        torch.cuda.synchronize()
        out[chunk] = (g, eng.actions_out.cpu().clone(), eng.rewards_out.cpu().clone(),
                      {k: v.cpu().clone() for k, v in eng.state.as_dict().items()}, eng.stat_slab.sum(0).cpu())
    g32, a32, r32, s32, st32 = out[32]
    g64, a64, r64, s64, st64 = out[64]
    assert torch.equal(a32, a64) and torch.equal(r32, r64)
    for k in s32:
        assert torch.equal(s32[k].nan_to_num(-1.0), s64[k].nan_to_num(-1.0)), k
    assert _rel(g64, g32) < 1e-4, _rel(g64, g32)
    assert torch.allclose(st64, st32, rtol=1e-4, atol=1e-3)


def test_bf16_gradient_slabs_match_fp32(native_built):
    """64-env-chunk kernel: bf16 per-workgroup gradient partials (the default) vs fp32 partials on
    the same state -- identical transitions, gradients equal up to one bf16 rounding per partial."""
    from sharetrade.trainer.engine import VectorEngine

    E = 4096
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    out = {}
    for sd in ("fp32", "bf16"):
        cfg = _cfg(False)
        cfg.agent.epsilon = 0.5
        cfg.engine.chunk = 64
        cfg.engine.slab_dtype = sd
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.slab_bf16 == (sd == "bf16")
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 5 % 150)
        eng.ctrl.fill_(7)
        g = eng.native_grad().detach().cpu().clone()
        torch.cuda.synchronize()
        out[sd] = (g, eng.actions_out.cpu().clone(), eng.stat_slab.sum(0).cpu())
    g32, a32, st32 = out["fp32"]
    g16, a16, st16 = out["bf16"]
    assert torch.equal(a32, a16)
    assert torch.equal(st32, st16)
    assert _rel(g16, g32) < 4e-3, _rel(g16, g32)
    assert _rel(g16, g32) > 0.0   # the bf16 path really ran


@pytest.mark.parametrize("opt", ["adam", "adagrad", "sgd"])
def test_optimizer_step_matches_reference(native_built, opt):
    from sharetrade.models import qnet as qn
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    cfg.agent.optimizer = opt
    cfg.agent.lr = 1e-2
    E = 64
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    p0 = eng.params.detach().cpu().clone()
    st = qn.OptimState(opt, eng.layout.numel, cfg.agent.adagrad_init_acc)
    for it in range(3):
        grad = eng.native_grad().detach().cpu().clone()
        # apply the native update only (mode 2 on the already-reduced grad)
        eng._op.mode = 2
        from sharetrade.ops import native

        native.check(native.lib().st_reduce_optim(eng._op, native.stream_handle()), "update")
        torch.cuda.synchronize()
        qn.optimizer_step_ref(p0, grad, st, eng.mask.cpu(), cfg.agent.lr, cfg.agent.adam_betas, cfg.agent.adam_eps)
        got = eng.params.detach().cpu()
        assert torch.allclose(got, p0, rtol=1e-5, atol=1e-6), (opt, it, float((got - p0).abs().max()))
        assert torch.equal(eng.params_bf.float().cpu(), got.to(torch.bfloat16).float())


def test_random_walk_kernel(native_built):
    from sharetrade.ops import native

    E, T = 256, 3000
    out = torch.empty(E, T, device="cuda")
    native.random_walk(out, 50.0, 0.02, 0.0, 123, 456)
    torch.cuda.synchronize()
    p = out.double().cpu()
    assert torch.isfinite(p).all() and (p > 0).all()
    assert torch.allclose(p[:, 0], torch.full((E,), 50.0, dtype=torch.float64), rtol=1e-6)
    r = torch.log(p[:, 1:] / p[:, :-1])
    assert abs(float(r.mean())) < 2e-3
    assert abs(float(r.std()) - 0.02) < 1e-3
    # rows differ, and the generator is deterministic
    assert not torch.equal(p[0], p[1])
    out2 = torch.empty_like(out)
    native.random_walk(out2, 50.0, 0.02, 0.0, 123, 456)
    assert torch.equal(out, out2)


def test_graph_replay_matches_eager(native_built):
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    E = 128
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    a = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    b = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    b.capture_graph(warmup=2)   # runs 2 eager steps + captures (no replay yet)
    a.run(2)
    for _ in range(5):
        a.step()
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state.budget, b.state.budget)
    assert torch.equal(a.state.pos, b.state.pos)
    assert int(a.ctrl[0]) == int(b.ctrl[0]) == 7


def test_multi_step_graph_matches_eager(native_built):
    """engine.graph_steps: run(n) replays k-step graphs then single steps -- bit-identical to n
    eager steps (the step index lives in device memory)."""
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    E = 128
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    a = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    b = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    b.capture_graph(warmup=2, graph_steps=4)
    a.run(2)
    a.run(11)          # no graph: 11 eager steps
    b.run(11)          # 2 x 4-step graph + 3 single-step replays
    torch.cuda.synchronize()
    assert a.step_count == b.step_count == 13
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state.budget, b.state.budget)
    assert torch.equal(a.state.pos, b.state.pos)
    assert int(a.ctrl[0]) == int(b.ctrl[0]) == 13


def test_compat_env_rewards_zero(native_built):
    """Quirk Q1 on the GPU path: decisions from constructor budget/shares => reward 0."""
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg(compat=True)
    cfg.env.features = "raw"
    E = 64
    eng = VectorEngine(cfg, prices=_prices(E, T=260), device=torch.device("cuda", 0), envs=E)
    eng.run(70)  # > one episode (T - H = 59 steps)
    torch.cuda.synchronize()
    s = eng.stats_dict()
    assert s["reward_sum"] == 0.0
    assert s["episodes_done"] == E
    fin = eng.final_portfolios().cpu()
    assert torch.all(fin == cfg.env.budget)


def test_dynamic_chunk_schedule_matches_static(native_built):
    """csrc/qstep_wide.hip dynamic schedule (per-XCD claim heads): every chunk is stepped exactly once
    per launch (positions advance by one, heads re-zeroed by the slab pass), transitions equal the
    static schedule's and gradients agree up to the bf16 rounding of differently-grouped partials."""
    from sharetrade.trainer.engine import VectorEngine

    E = 64 * 8 * 6   # 48 chunks over a grid of 16: 3 per workgroup on average
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    out = {}
    for sched in ("static", "dynamic"):
        cfg = _cfg(False)
        cfg.agent.epsilon = 0.5
        cfg.engine.chunk = 64
        cfg.engine.chunk_schedule = sched
        cfg.engine.grid = 16
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.chunk_schedule == sched and eng.grid == 16
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 5 % 150)
        pos0 = eng.state.pos.clone()
        eng.ctrl.fill_(7)
        g = eng.native_grad().detach().cpu().clone()
        torch.cuda.synchronize()
        assert torch.equal(eng.state.pos, pos0 + 1), "a chunk was skipped or stepped twice"
        out[sched] = (g, eng.actions_out.cpu().clone(), eng.stat_slab.sum(0).cpu())
        if sched == "dynamic":
            assert int(eng.chunk_heads.abs().sum()) == 0, "claim heads not re-zeroed"
            g2 = eng.native_grad().detach().cpu().clone()   # second launch: heads reset worked
            torch.cuda.synchronize()
            assert torch.equal(eng.state.pos, pos0 + 2)
            assert torch.isfinite(g2).all()
    gs, as_, sts = out["static"]
    gd, ad, std_ = out["dynamic"]
    assert torch.equal(ad, as_)
    assert _rel(gd, gs) < 4e-3, _rel(gd, gs)
    assert torch.allclose(std_, sts, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("chunk", [32, 64])
def test_reward_modes_and_td_clip_match_oracle(native_built, chunk):
    """agent.reward_mode = relative / absolute and agent.td_clip (Huber) in both step kernels vs the
    torch oracle: identical rewards and transitions, gradients within the bf16 tolerance."""
    from sharetrade.env import trading as tr
    from sharetrade.trainer.engine import VectorEngine

    E = 128
    prices = _prices(E)
    dev = torch.device("cuda", 0)
    for mode, clip in (("absolute", 0.0), ("relative", 0.0), ("absolute", 0.5)):
        cfg = _cfg(False)
        cfg.agent.epsilon = 0.5
        cfg.agent.reward_mode, cfg.agent.td_clip = mode, clip
        cfg.engine.chunk = chunk
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.chunk == chunk
        eng.state.pos.copy_(torch.arange(E, dtype=torch.int32, device=dev) * 3 % 150)
        eng.state.shares.copy_(torch.arange(E, dtype=torch.int32, device=dev) % 3)
        eng.state.value.copy_(prices[:, 0].to(dev))
        st0 = eng.state.clone().to("cpu")
        eng.ctrl.fill_(5)
        params = eng.params.detach().cpu().clone()
        grad = eng.native_grad().detach().cpu().clone()
        torch.cuda.synchronize()
        acts, rew = eng.actions_out.cpu().clone(), eng.rewards_out.cpu().clone()
        ns, g_ref, info = tr.engine_step_ref(
            prices, st0, params, eng.layout, history=cfg.model.history, feature_mode=cfg.env.features,
            budget0=cfg.env.budget, shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions,
            target_slot=cfg.agent.target_slot, gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu,
            epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=5,
            loss_coef=eng.loss_coef, reward_mode=mode, td_clip=clip, emulate_bf16=True, forced_actions=acts)
        assert torch.equal(info["reward"], rew), mode
        if mode == "relative":
            assert float(rew.abs().max()) < 0.5   # one-step returns, not dollars
        for k in ("budget", "shares", "value", "pos"):
            assert torch.equal(getattr(ns, k), getattr(eng.state, k).cpu()), (mode, k)
        assert _rel(grad, g_ref) < 3e-2, (mode, clip, _rel(grad, g_ref))


@pytest.mark.parametrize("kernel,E,bank16", [("wide", 131072, "auto"), ("ws", 393216, "off"), ("ws", 786432, "auto")])
def test_large_bank_gather_matches_oracle(native_built, kernel, E, bank16):
    """x 6,047 days: the wide kernel's 4 aligned replicas of 131,072 envs hold 3.2e9 floats, the ws
    kernel's single padded copy of 393,216 envs 2.4e9, so the window offsets of the upper envs pass
    2^31 elements (the bench runs 1,835,008 envs per GPU).  The last 512 envs (windows spread over the
    whole series) must select the same greedy actions as the fp32 oracle on their own rows and make
    bit-identical env transitions."""
    from sharetrade.env import trading as tr
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    cfg.agent.epsilon, cfg.agent.ramp = 1.0, 1.0   # exploit whenever pos >= 1: actions = argmax Q(x)
    cfg.data.source, cfg.data.length = "random_walk", 6047
    cfg.engine.step_kernel = kernel
    cfg.engine.bank16 = bank16
    S = 512
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, envs=E)
    assert eng.chunk == 64 and eng.step_kernel == kernel
    if kernel == "ws" and bank16 == "auto":
        # the synthetic bank is on a tick grid: the ws windows come from the 16-bit tick copy (4.8e9 ticks)
        assert eng.prices4 is None and eng.ticks.numel() > 2 ** 32
    else:
        assert eng.ticks is None and eng.prices4.numel() > 2 ** 31
        assert eng.prices4.shape[0] == (1 if kernel == "ws" else 4)
    idx = torch.arange(E, dtype=torch.int32, device=dev)
    eng.state.pos.copy_(1 + idx * 37 % (eng.T - cfg.model.history - 3))
    eng.state.shares.copy_(idx % 3)
    eng.state.value.copy_(eng.prices[:, 0])
    st0 = eng.state.clone()
    eng.ctrl.fill_(5)
    params = eng.params.detach().cpu().clone()
    eng.native_grad()
    torch.cuda.synchronize()
    sub = slice(E - S, E)
    acts = eng.actions_out[sub].cpu().clone()
    prices = eng.prices[sub].cpu().clone()
    st_sub = tr.EnvState(**{k: v[sub].cpu().clone() for k, v in st0.as_dict().items()})
    kw = dict(history=cfg.model.history, feature_mode=cfg.env.features, budget0=cfg.env.budget,
              shares0=cfg.env.shares, compat_env=cfg.env.compat_decisions, target_slot=cfg.agent.target_slot,
              gamma=cfg.agent.gamma, output_relu=cfg.model.output_relu, epsilon=cfg.agent.epsilon,
              ramp=cfg.agent.ramp, seed=cfg.agent.seed, rank=0, step=5, loss_coef=eng.loss_coef,
              env_offset=E - S, reward_mode=cfg.agent.reward_mode, td_clip=cfg.agent.td_clip, emulate_bf16=True)
    _, _, info0 = tr.engine_step_ref(prices, st_sub, params, eng.layout, **kw)
    assert bool(info0["exploit"].all())
    mism = (info0["actions"].cpu() != acts).float().mean().item()
    assert mism <= 0.05, f"action mismatch rate {mism}"
    ns, _, info = tr.engine_step_ref(prices, st_sub, params, eng.layout, forced_actions=acts, **kw)
    assert torch.equal(info["reward"], eng.rewards_out[sub].cpu())
    for k in ("budget", "shares", "value", "pos"):
        assert torch.equal(getattr(ns, k), getattr(eng.state, k)[sub].cpu()), k


def test_graph_priming_is_rank_uniform(native_built):
    """prime_graph: one process stops once two consecutive replays agree; with world_size > 1 it
    replays exactly min_reps times on every rank (each replay holds the DP all-reduce, so a
    per-rank stopping decision could leave ranks with different collective counts)."""
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg(False)
    cfg.engine.graph_steps = 4
    eng = VectorEngine(cfg, prices=_prices(256), device=torch.device("cuda", 0), envs=256)
    assert eng.capture_graph(warmup=1, prime=True, prime_reps=2)
    s0 = eng.step_count
    n = eng.prime_graph(3)
    assert 3 <= n <= 40 and eng.step_count == s0 + 4 * n
    eng.world_size = 2          # only the stopping rule is exercised (no collective in this graph)
    s1 = eng.step_count
    assert eng.prime_graph(5) == 5 and eng.step_count == s1 + 20
    eng.world_size = 1
    # bench.py's fixed priming (max_reps = min_reps): exactly that many replays on one process too
    s2 = eng.step_count
    assert eng.prime_graph(6, max_reps=6) == 6 and eng.step_count == s2 + 24
