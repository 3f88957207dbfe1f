"""Numerics of the batched serving kernel (``csrc/qserve.hip``) vs the fp32 PyTorch oracle.

The oracle (``sharetrade.serve.reference_select``) rounds the features and hidden activations to
bf16 where the kernel does; only the fp32 accumulation order differs, so Q values are compared with
a tight relative tolerance and actions must agree wherever the top-two Q margin is not a near-tie.
The epsilon-greedy draws use the same Philox counters on both sides.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rows(B, H=201, seed=0):
    g = np.random.default_rng(seed)
    p = 50.0 * np.exp(np.cumsum(g.normal(0, 0.02, size=(B, H)), axis=1))
    budget = g.uniform(0, 5000, size=(B, 1))
    shares = g.integers(0, 40, size=(B, 1)).astype(np.float64)
    return torch.from_numpy(np.concatenate([p, budget, shares], 1).astype(np.float32))


def _cfg(features="relative", output_relu=False):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship")
    cfg.env.features = features
    cfg.model.output_relu = output_relu
    if features == "raw":
        cfg.model.init_std = 0.01
        cfg.model.init = "normal"
    return cfg


def _check(srv, x, steps, seq):
    from sharetrade.serve import reference_select

    c = srv.cfg
    a, q = srv.infer(x, steps, return_q=True)
    a_ref, q_ref = reference_select(srv.params, srv.layout, x.cuda(), history=srv.H, feat_mode=c.env.features,
                                    output_relu=c.model.output_relu, budget0=c.env.budget,
                                    epsilon=c.agent.epsilon, ramp=c.agent.ramp, key_seed=srv.seed, seq=seq,
                                    steps=steps)
    rel = float((q - q_ref).norm() / (q_ref.norm() + 1e-12))
    assert rel < 2e-3, rel
    top2 = q_ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3 * (q_ref.abs().max(1).values + 1e-3)
    assert clear.float().mean() > 0.5
    assert torch.equal(a[clear], a_ref[clear])


@pytest.mark.parametrize("B", [1, 63, 64, 1000, 70001])
def test_serve_kernel_matches_oracle(native_built, B):
    from sharetrade.serve import PolicyServer

    srv = PolicyServer(_cfg(), device=torch.device("cuda", 0), backend="native")
    assert srv.backend == "native"
    x = _rows(B, seed=B)
    _check(srv, x, None, 0)                      # greedy (seq 0)
    steps = torch.from_numpy(np.random.default_rng(B).uniform(0, 2000, size=B).astype(np.float32))
    _check(srv, x, steps, 1)                     # epsilon-greedy draws of batch 1


@pytest.mark.parametrize("features,output_relu", [("raw", True), ("raw", False), ("relative", True)])
def test_serve_kernel_feature_modes(native_built, features, output_relu):
    from sharetrade.serve import PolicyServer

    srv = PolicyServer(_cfg(features, output_relu), device=torch.device("cuda", 0), backend="native")
    _check(srv, _rows(300, seed=7), None, 0)


def test_serve_kernel_strided_rows_and_engine_weights(native_built):
    """Rows read with their own stride (a wider buffer), weights taken from a training engine."""
    from sharetrade.serve import PolicyServer, reference_select
    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    cfg.engine.envs_per_rank = 256
    eng = VectorEngine(cfg, device=torch.device("cuda", 0))
    eng.run(3)
    srv = PolicyServer.from_engine(eng)
    wide = torch.zeros(500, 256)
    wide[:, :203] = _rows(500, seed=11)
    a, q = srv.infer(wide[:, :203], return_q=True)   # non-contiguous view -> copied rows
    a_ref, q_ref = reference_select(eng.params, srv.layout, wide[:, :203].cuda(), history=201,
                                    feat_mode="relative", output_relu=False, budget0=cfg.env.budget,
                                    epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, key_seed=srv.seed)
    assert float((q - q_ref).norm() / q_ref.norm()) < 2e-3
    # strided launch straight from the wide buffer
    dev_wide = wide.cuda()
    acts = torch.empty(500, dtype=torch.int32, device="cuda")
    q2 = torch.empty(500, 3, device="cuda")
    srv._kern.launch(dev_wide[:, :203], acts, q2)
    assert torch.equal(q2, q) and torch.equal(acts, a)


def test_batcher_native_path(native_built):
    import threading

    from sharetrade.serve import DynamicBatcher, PolicyServer

    srv = PolicyServer(_cfg(), device=torch.device("cuda", 0), backend="native")
    x = _rows(300, seed=5)
    want = srv.infer(x).cpu().tolist()
    out = [None] * 300
    with DynamicBatcher(srv, max_batch=128, max_delay_us=5000, greedy=True) as bat:
        def client(lo, hi):
            fs = [(i, bat.submit(x[i])) for i in range(lo, hi)]
            for i, f in fs:
                out[i] = f.result(timeout=60)

        ts = [threading.Thread(target=client, args=(k * 100, (k + 1) * 100)) for k in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert out == want


def test_aligned_and_unaligned_gathers_agree(native_built):
    """Rows at stride 203 (dword gather) and at the server's aligned stride 204 (dwordx4 gather)."""
    from sharetrade.serve import PolicyServer

    srv = PolicyServer(_cfg(), device=torch.device("cuda", 0), backend="native")
    x = _rows(777, seed=13)
    a, q = srv.infer(x, torch.full((777,), 700.0), return_q=True)   # aligned staging, batch seq 0
    xd = x.cuda().contiguous()
    assert xd.stride(0) == 203
    a2 = torch.empty(777, dtype=torch.int32, device="cuda")
    q2 = torch.empty(777, 3, device="cuda")
    srv._kern.launch(xd, a2, q2, torch.full((777,), 700.0, device="cuda"), seq=0)
    assert torch.equal(q2, q) and torch.equal(a2, a)


def test_http_front_end_native(native_built):
    from fastapi.testclient import TestClient

    from sharetrade.serve import DynamicBatcher, PolicyServer
    from sharetrade.serve.http import make_app

    srv = PolicyServer(_cfg(), device=torch.device("cuda", 0), backend="native")
    x = _rows(9, seed=21)
    want = srv.infer(x).cpu().tolist()
    with DynamicBatcher(srv, max_batch=32, max_delay_us=500, greedy=True) as bat:
        c = TestClient(make_app(srv, bat))
        r = c.post("/select", json={"states": x.tolist()})
        assert r.status_code == 200 and r.json()["actions"] == want
        r = c.post("/selection_action", json={"current_state": x[4].tolist(), "step": 0.0})
        assert r.status_code == 200 and r.json()["index"] == want[4]   # greedy batcher
        import numpy as np

        body = np.concatenate([x.numpy(), np.full((9, 1), -1.0, np.float32)], 1).astype("<f4").tobytes()
        r = c.post("/select_bin", content=body)   # binary rows, greedy
        assert r.status_code == 200 and [int(v) for v in np.frombuffer(r.content, np.int8)] == want
        assert c.get("/health").json()["backend"] == "native"


def test_optimizer_kernel_polyak_average(native_built):
    """csrc/optim.hip advances ema <- ema + (1 - d)(w - ema) in the optimizer pass: bit-equal to the host
    recurrence over the engine's parameter trajectory, eager and inside captured graphs."""
    import numpy as np

    from sharetrade.trainer.engine import VectorEngine

    cfg = _cfg()
    cfg.engine.ema_decay = 0.95
    eng = VectorEngine(cfg, device=torch.device("cuda", 0), envs=256)
    c = float(np.float32(1.0) - np.float32(0.95))
    want = eng.params.clone()
    for _ in range(3):
        eng.step()
        torch.cuda.synchronize()
        want = want + (eng.params - want) * c
    assert torch.equal(eng.params_ema, want)
    assert eng.capture_graph(warmup=0, graph_steps=2)
    p_before = eng.params.clone()
    eng.run(1)   # one single-step graph replay
    torch.cuda.synchronize()
    want = want + (eng.params - want) * c
    assert not torch.equal(p_before, eng.params) and torch.equal(eng.params_ema, want)
