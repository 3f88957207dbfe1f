"""Learning-quality experiment knobs (agent.target_every / double_dqn / reward_scale / ramp_mode) on the torch
backend (tools/learning_eval.py --backend torch; the native batched fp32 step is pinned to it by
tests/test_gpu_f32.py::test_fp32_batched_learning_knobs_match_torch_engine).  The reference bootstraps Q(x') from the online net with
the exploit ramp over the episode position (QDecisionPolicyActor.scala:58-71); these runs test whether a
target network, Double DQN, a larger reward scale or a ramp annealed over training help the learned policy."""
import numpy as np
import pytest
import torch

from sharetrade.config import preset_config
from sharetrade.data.prices import random_walk
from sharetrade.trainer.engine import VectorEngine


def _eng(**agent):
    cfg = preset_config("flagship")
    for k, v in agent.items():
        setattr(cfg.agent, k, v)
    E, T = 64, 240
    prices = torch.from_numpy(random_walk(T, 50.0, 0.02, 3, n_series=E).astype(np.float32))
    return VectorEngine(cfg, prices=prices, device=torch.device("cpu"), envs=E, backend="torch")


def test_defaults_match_plain_step():
    a, b = _eng(), _eng(reward_scale=1.0, ramp_mode="position")
    for _ in range(3):
        a.step()
        b.step()
    assert torch.equal(a.params, b.params)


def test_target_network_refresh_and_snapshot():
    e = _eng(target_every=2, target_slot="action")
    e.step()
    t1 = e.params_target.clone()
    assert not torch.equal(t1, e.params)            # not refreshed after step 1
    e.step()
    assert torch.equal(e.params_target, e.params)   # refreshed after step 2
    d = e.state_dict()
    e.step()
    e.load_state_dict(d)
    assert torch.equal(e.params_target, d["params_target"])


def test_target_and_double_dqn_change_the_update():
    base, tgt, dd = _eng(target_slot="action"), _eng(target_every=50, target_slot="action"), \
        _eng(target_every=50, double_dqn=True, target_slot="action")
    for e in (base, tgt, dd):
        for _ in range(3):
            e.step()
    assert not torch.equal(base.params, tgt.params)
    assert not torch.equal(tgt.params, dd.params)


def test_global_ramp_and_reward_scale():
    a, b = _eng(ramp_mode="global", ramp=2.0), _eng(reward_scale=100.0)
    ref = _eng()
    for e in (a, b, ref):
        for _ in range(3):
            e.step()
    assert not torch.equal(a.params, ref.params) and not torch.equal(b.params, ref.params)


def test_double_dqn_needs_a_target_net():
    # (the bf16 native step takes the knobs on the ws kernel only: tests/test_gpu_ws_knobs.py)
    cfg = preset_config("flagship")
    cfg.agent.double_dqn = True
    with pytest.raises(ValueError):
        VectorEngine(cfg, device=torch.device("cpu"), envs=64, backend="torch")


def test_f32_deterministic_auto_policy(monkeypatch):
    """engine.f32_deterministic='auto': ordered partial sums (bit-reproducible) for DP ranks and for the
    reference's decision semantics; fp32 atomics for a single 'intended' process; the env override wins."""
    from sharetrade.ops.mlp_f32 import f32_deterministic

    monkeypatch.delenv("SHARETRADE_F32_SPLIT_PARTIAL", raising=False)
    ref, intended = preset_config("reference_compat"), preset_config("intended")
    assert f32_deterministic(ref, 1) and f32_deterministic(intended, 2) and not f32_deterministic(intended, 1)
    intended.engine.f32_deterministic = "on"
    assert f32_deterministic(intended, 1)
    ref.engine.f32_deterministic = "off"
    assert not f32_deterministic(ref, 4)
    monkeypatch.setenv("SHARETRADE_F32_SPLIT_PARTIAL", "1")
    assert f32_deterministic(ref, 4)
    intended.engine.f32_deterministic = "sometimes"
    monkeypatch.delenv("SHARETRADE_F32_SPLIT_PARTIAL")
    with pytest.raises(ValueError):
        f32_deterministic(intended, 1)


def test_flagship_stable_preset_runs_the_knobs():
    """preset flagship_stable = flagship + target net / Double DQN / reward scale / global ramp; the torch
    engine steps it (the native ws path is pinned on the GPU: tests/test_gpu_ws_knobs.py)."""
    cfg = preset_config("flagship_stable")
    a = cfg.agent
    assert (a.target_every, a.double_dqn, a.reward_scale, a.ramp_mode, a.gamma) == (1000, True, 100.0, "global", 0.99)
    assert cfg.model.hidden == preset_config("flagship").model.hidden
    e = VectorEngine(cfg, device=torch.device("cpu"), envs=8, backend="torch")
    for _ in range(2):
        e.step()
    assert e.params_target is not None and torch.isfinite(e.params).all()
