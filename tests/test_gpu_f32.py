"""Exact-fp32 HIP kernels (csrc/mlp_f32.hip) vs the plain-PyTorch fp32 oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture
def dev(native_built):
    return torch.device("cuda", 0)


def _states(B, seed=0, raw=True):
    rng = np.random.default_rng(seed)
    x = rng.uniform(15, 180, (B, 203)).astype(np.float32)
    if raw:
        x[:, 201] = rng.uniform(500, 2400, B)
        x[:, 202] = rng.integers(0, 5, B)
    return torch.from_numpy(x)


@pytest.mark.parametrize("preset", ["reference_compat", "intended", "flagship"])
def test_forward_matches_oracle(dev, preset):
    from sharetrade.config import preset_config
    from sharetrade.models import qnet as qn
    from sharetrade.policy.learner import QLearner

    cfg = preset_config(preset)
    ln = QLearner(cfg, device=dev)
    assert ln.backend == "native"
    x = _states(9, raw=preset != "flagship")
    got = ln.q_values(x).cpu()
    ref, _, _ = qn.forward(ln.params.cpu(), ln.layout, x, cfg.model.output_relu)
    assert torch.allclose(got, ref[:, :3], rtol=2e-5, atol=1e-3 * float(ref.abs().max() + 1)), (got, ref[:, :3])


@pytest.mark.parametrize("opt", ["adagrad", "adam", "sgd"])
@pytest.mark.parametrize("slot", ["compat", "action"])
@pytest.mark.parametrize("B", [1, 5])
def test_td_update_matches_oracle(dev, opt, slot, B):
    from sharetrade.config import preset_config
    from sharetrade.policy.learner import QLearner

    cfg = preset_config("intended" if slot == "action" else "reference_compat")
    cfg.agent.optimizer = opt
    cfg.agent.lr = 1e-3 if opt != "sgd" else 1e-5
    cfg.agent.target_slot = slot
    cpu = QLearner(cfg, device=torch.device("cpu"))
    # same starting weights (the device init kernel matches the host mirror only up to libm ulps:
    # test_init_normal_kernel_matches_host_mirror)
    gpu = QLearner(cfg, device=dev, params=cpu.params)
    assert torch.equal(gpu.params.cpu(), cpu.params)
    for it in range(3):
        x, xn = _states(B, 10 + it) / 100.0, _states(B, 20 + it) / 100.0
        r = np.linspace(-3, 3, B).astype(np.float32)
        acts = np.arange(B) % 3 if slot == "action" else None
        lg = gpu.update(x, r, xn, acts)
        lc = cpu.update(x, r, xn, acts)
        assert abs(lg - lc) <= 1e-4 * max(1.0, abs(lc)), (lg, lc)
        assert _rel(gpu.params.cpu(), cpu.params) < 1e-5, _rel(gpu.params.cpu(), cpu.params)
        if cpu.opt.s1.numel():
            assert _rel(gpu.opt.s1.cpu(), cpu.opt.s1) < 1e-4


@pytest.mark.parametrize("B", [1, 3])
def test_staged_host_inputs_match_device_inputs(dev, B):
    """Host inputs go through the pinned staging image (one H2D copy); device inputs through the
    pad path: identical parameters, Q values and losses; ``return_loss=False`` defers the read-back."""
    from sharetrade.config import preset_config
    from sharetrade.policy.learner import QLearner

    cfg = preset_config("intended")
    a, b = QLearner(cfg, device=dev), QLearner(cfg, device=dev)
    for it in range(4):
        x, xn = _states(B, 30 + it) / 100.0, _states(B, 40 + it) / 100.0
        r = np.linspace(-1, 2, B).astype(np.float32)
        acts = (np.arange(B) + it) % 3
        la = a.update(x, r, xn, acts, return_loss=False)
        assert la is None
        lb = b.update(torch.as_tensor(x, device=dev), r, torch.as_tensor(xn, device=dev), acts)
        assert a.last_loss == lb
    assert torch.equal(a.params, b.params)
    q_host = a.q_values(x)
    q_dev = a.q_values(torch.as_tensor(x, device=dev))
    assert torch.equal(q_host, q_dev)


def test_policy_actor_on_gpu_uses_native_learner(dev):
    from sharetrade import protocol as P
    from sharetrade.actors.runtime import ActorSystem
    from sharetrade.config import preset_config
    from sharetrade.policy.actor import QDecisionPolicyActor

    s = ActorSystem("gpu")
    try:
        pol = s.actor_of(QDecisionPolicyActor.props(preset_config("test"), device=dev))
        st = list(range(55, 256)) + [1000, 0]
        nx = list(range(55, 256)) + [940, 1]
        assert pol.ask(P.UpdateQ(st, 10.0, nx), 10).result(20) is P.Updated
        assert isinstance(pol.ask(P.SelectionAction(st, 0), 10).result(20), P.Action)
        actor = pol._cell.actor
        assert actor.learner.backend == "native"
    finally:
        s.terminate()


@pytest.mark.parametrize("preset", ["reference_compat", "intended"])
def test_fp32_engine_matches_torch_engine(dev, preset):
    """The fp32 engine step (rows kernel + grad/optim) vs the oracle engine for 6 steps."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config(preset)
    cfg.engine.dtype = "fp32"
    cfg.agent.epsilon = 0.5
    cfg.agent.ramp = 4.0          # exploit early so argmax paths are exercised
    E, T = 10, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 5, n_series=E).astype(np.float32))
    g = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    c = VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")
    assert g.kernel == "fp32_rows"
    for _ in range(6):
        g.step()
        c.step()
        torch.cuda.synchronize()
        for k in ("budget", "shares", "pos"):
            assert torch.equal(getattr(g.state, k).cpu(), getattr(c.state, k)), k
        assert _rel(g.params.cpu(), c.params) < 1e-5


def test_fp32_engine_compat_reproduces_reference_portfolio(dev):
    """Quirk Q1 on the GPU fp32 path: reward 0 at every step, final portfolio = budget."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("reference_compat")
    E, T = 10, 320
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 9, n_series=1).astype(np.float32)).expand(E, -1)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    eng.capture_graph(warmup=1) if hasattr(eng, "capture_graph") else None
    eng.run(T - 201 - 1)
    torch.cuda.synchronize()
    assert float(eng.stat_acc[0]) == 0.0
    fin = eng.final_portfolios().cpu()
    assert torch.all(fin == 2400.0), fin


def test_init_normal_kernel_matches_host_mirror(native_built):
    """The device init kernel (csrc/series.hip, Philox + Box-Muller) vs its NumPy mirror: the same
    counters, so the same normals up to device-vs-libm transcendental ulps."""
    import torch

    from sharetrade.config import preset_config
    from sharetrade.models import qnet as qn

    for preset in ("reference_compat", "flagship"):
        cfg = preset_config(preset)
        L = qn.QNetLayout.from_config(cfg.model)
        host = qn.init_params(L, cfg.model, seed=5, host_mirror=True)   # the NumPy mirror, not the kernel
        dev = qn.init_params(L, cfg.model, seed=5, device="cuda:0").cpu()
        assert torch.equal(dev == 0, host == 0)                 # same padding pattern
        assert torch.allclose(dev, host, rtol=2e-5, atol=2e-6), float((dev - host).abs().max())


@pytest.mark.parametrize("preset", ["reference_compat", "intended"])
def test_fp32_batched_engine_matches_torch_engine(dev, preset):
    """The batched fp32 MFMA step (csrc/mlp_f32_mfma.hip, the reference's 203->200->3 net over 1,024 envs)
    vs the plain-PyTorch fp32 oracle engine for 5 steps: the same env transitions, parameters within
    fp32 summation-order tolerance."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config(preset)
    cfg.engine.dtype = "fp32"
    cfg.agent.epsilon = 0.5
    cfg.agent.ramp = 4.0
    E, T = 1024, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 5, n_series=E).astype(np.float32))
    g = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    c = VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")
    assert g.kernel == "fp32_rows" and g.f32_path == "batched"
    for _ in range(5):
        g.step()
        c.step()
        torch.cuda.synchronize()
        for k in ("budget", "shares", "pos"):
            assert torch.equal(getattr(g.state, k).cpu(), getattr(c.state, k)), k
        assert _rel(g.params.cpu(), c.params) < 1e-5, _rel(g.params.cpu(), c.params)


@pytest.mark.parametrize("preset", ["reference_compat", "intended"])
def test_fp32_batched_matches_row_kernels(dev, preset):
    """Batched MFMA step vs the per-env row kernels on the same engine state (uniform actions): equal
    transitions, gradients equal up to fp32 summation order, in captured graphs."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    E, T = 2048, 300
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 8, n_series=E).astype(np.float32))
    out = {}
    for path in ("on", "off"):
        cfg = preset_config(preset)
        cfg.engine.dtype = "fp32"
        cfg.engine.f32_batched = path
        cfg.agent.epsilon = 0.0
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng.f32_path == ("batched" if path == "on" else "rows")
        g = eng.native_grad().detach().cpu().clone()
        eng.capture_graph(warmup=1)
        eng.run(6)
        torch.cuda.synchronize()
        out[path] = (g, eng.params.cpu().clone(), {k: v.cpu().clone() for k, v in eng.state.as_dict().items()})
    (gb, pb, sb), (gr, pr, sr) = out["on"], out["off"]
    # reference_compat's reward is 0 (quirk Q1), so its gradient is a sum of +/- TD terms over 2,048 envs
    # that nearly cancel: the batched path's split-K atomics and the rows path's fixed-order reduction
    # then differ by ~1e-4 of the (small) result; intended's gradient does not cancel
    tol = 1e-3 if preset == "reference_compat" else 1e-5
    assert _rel(gb, gr) < tol, _rel(gb, gr)
    for k in ("budget", "shares", "pos", "value"):
        assert torch.equal(sb[k], sr[k]), k
    assert _rel(pb, pr) < 1e-5, _rel(pb, pr)


def test_fp32_batched_compat_reproduces_reference_portfolio(dev):
    """Quirk Q1 through the batched path: 1,024 envs of the reference run, reward 0, every final
    portfolio exactly the 2,400 budget."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("reference_compat")
    E, T = 1024, 320
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 9, n_series=1).astype(np.float32)).expand(E, -1)
    eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    assert eng.f32_path == "batched"
    eng.capture_graph(warmup=1)
    eng.run(T - 201 - 1)
    torch.cuda.synchronize()
    assert float(eng.stat_acc[0]) == 0.0
    fin = eng.final_portfolios().cpu()
    assert torch.all(fin == 2400.0), fin


@pytest.mark.parametrize("preset", ["reference_compat", "intended"])
def test_fp32_fused_forward_matches_two_gemm_forward(dev, preset, monkeypatch):
    """From 8,192 envs the batched step's forward is one launch (csrc/mlp_f32_mfma.hip f32b_fwd2_kernel:
    hidden layer on 64 x 256 tiles, the 3-action output from registers); vs the two-GEMM forward
    (SHARETRADE_F32_FWD2=0) over 4 captured steps: same transitions, Q / H / parameters within fp32
    summation-order tolerance."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    E, T = 8192, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 11, n_series=E).astype(np.float32))
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("SHARETRADE_F32_FWD2", fused)
        cfg = preset_config(preset)
        cfg.engine.dtype = "fp32"
        cfg.engine.f32_batched = "on"
        cfg.agent.epsilon = 0.5
        cfg.agent.ramp = 4.0
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert eng._f32._fwd2_ok() == (fused == "1")
        eng.capture_graph(warmup=1)
        eng.run(4)
        torch.cuda.synchronize()
        s = eng._f32.s
        out[fused] = (s.q.cpu().clone(), s.A[1].cpu().clone(), eng.params.cpu().clone(),
                      {k: v.cpu().clone() for k, v in eng.state.as_dict().items()})
    (qf, hf, pf, sf), (qg, hg, pg, sg) = out["1"], out["0"]
    for k in ("budget", "shares", "pos", "value"):
        assert torch.equal(sf[k], sg[k]), k
    assert _rel(hf, hg) < 1e-5, _rel(hf, hg)
    assert _rel(qf, qg) < 1e-5, _rel(qf, qg)
    assert _rel(pf, pg) < 1e-5, _rel(pf, pg)
    assert torch.all(qf[:, 3:] == 0)


@pytest.mark.parametrize("preset,knobs", [
    ("intended", dict(target_every=2, double_dqn=True, reward_scale=10.0, ramp_mode="global")),
    ("intended", dict(target_every=3)),
    ("reference_compat", dict(target_every=2, reward_scale=4.0)),
])
def test_fp32_batched_learning_knobs_match_torch_engine(dev, preset, knobs):
    """Target network (refreshed on the device every target_every steps), Double DQN, reward scale and the
    exploit ramp over the step count on the batched fp32 step vs the torch oracle engine (engine_step_ref):
    same transitions, parameters and target parameters within fp32 summation-order tolerance over 5 steps."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config(preset)
    cfg.engine.dtype = "fp32"
    cfg.agent.epsilon = 0.5
    cfg.agent.ramp = 4.0
    for k, v in knobs.items():
        setattr(cfg.agent, k, v)
    if preset == "intended":
        cfg.agent.target_slot = "action"
    E, T = 1024, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 5, n_series=E).astype(np.float32))
    g = VectorEngine(cfg, prices=prices, device=dev, envs=E)
    c = VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")
    assert g.f32_path == "batched"
    for _ in range(5):
        g.step()
        c.step()
        torch.cuda.synchronize()
        for k in ("budget", "shares", "pos"):
            assert torch.equal(getattr(g.state, k).cpu(), getattr(c.state, k)), k
        assert _rel(g.params.cpu(), c.params) < 1e-5, _rel(g.params.cpu(), c.params)
        if knobs.get("target_every"):
            assert _rel(g.params_target.cpu(), c.params_target) < 1e-5


def test_fp32_batched_split_partials_match_atomics(dev, monkeypatch):
    """Weight gradients of the batched step with split-K partial tiles + one ordered sum
    (SHARETRADE_F32_SPLIT_PARTIAL=1, bit-reproducible) vs the default fp32 atomics: equal up to fp32
    summation order, and two partial-sum runs bit-identical."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    E, T = 8192, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 13, n_series=E).astype(np.float32))
    grads, wsl = {}, []
    for mode in ("partial", "partial2", "atomic"):
        monkeypatch.setenv("SHARETRADE_F32_SPLIT_PARTIAL", "0" if mode == "atomic" else "1")
        cfg = preset_config("intended")
        cfg.engine.dtype = "fp32"
        cfg.engine.f32_batched = "on"
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert (eng._f32.partials is None) == (mode == "atomic")
        grads[mode] = eng.native_grad().detach().cpu().clone()
        net, pd = eng._f32.net, eng.layout.pdims
        wsl = [slice(net.off_w[l], net.off_w[l] + pd[l + 1] * pd[l]) for l in range(eng.layout.n_layers)]
    for w in wsl:
        assert torch.equal(grads["partial"][w], grads["partial2"][w])
    # and the bias column sums (per-block partials + ordered sum): the whole gradient is bit-reproducible
    assert torch.equal(grads["partial"], grads["partial2"])
    assert _rel(grads["partial"], grads["atomic"]) < 1e-5, _rel(grads["partial"], grads["atomic"])


@pytest.mark.parametrize("hidden", [[512], [520, 300]])
def test_fp32_batched_deterministic_wide_layers(dev, monkeypatch, hidden):
    """Deterministic mode (engine.f32_deterministic: on for every DP rank and for reference_compat) on layers
    wider than the 256-column float4 bias sum, with biases trained: the ordered fallback sums (one partial row
    per 256 envs, st_f32b_splitsum's one-element form) instead of an error on the first step.  Two runs are
    bit-identical and agree with the fp32-atomic mode up to summation order."""
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.engine import VectorEngine

    E, T = 4096, 260
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 17, n_series=E).astype(np.float32))
    grads = {}
    for mode in ("det", "det2", "atomic"):
        monkeypatch.delenv("SHARETRADE_F32_SPLIT_PARTIAL", raising=False)
        cfg = preset_config("intended")
        cfg.model.hidden = list(hidden)
        cfg.model.train_bias = True
        cfg.engine.dtype = "fp32"
        cfg.engine.f32_batched = "on"
        cfg.engine.f32_deterministic = "off" if mode == "atomic" else "on"
        eng = VectorEngine(cfg, prices=prices, device=dev, envs=E)
        assert (eng._f32.partials is None) == (mode == "atomic")
        grads[mode] = eng.native_grad().detach().cpu().clone()
        eng.step()   # and a whole step (gradient -> optimizer) runs
        torch.cuda.synchronize()
        assert torch.isfinite(eng.params).all()
    assert torch.equal(grads["det"], grads["det2"])
    assert _rel(grads["det"], grads["atomic"]) < 1e-5, _rel(grads["det"], grads["atomic"])
