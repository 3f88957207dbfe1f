"""Policy serving on the CPU backend: server, dynamic batcher and the SelectionAction actor.

The GPU kernel itself is checked against the same oracle in ``tests/test_gpu_serve.py``.
"""
import threading

import numpy as np
import pytest
import torch

from sharetrade import protocol as P
from sharetrade.actors.runtime import ActorSystem
from sharetrade.actors.testkit import EventFilter, TestKit
from sharetrade.config import preset_config
from sharetrade.errors import IllegalArgumentException
from sharetrade.models import qnet as qn
from sharetrade.serve import (DynamicBatcher, LoadPolicy, PolicyLoaded, PolicyServer, PolicyServingActor,
                              reference_select)


def _rows(B, H=201, seed=0):
    g = np.random.default_rng(seed)
    p = 50.0 * np.exp(np.cumsum(g.normal(0, 0.02, size=(B, H)), axis=1))
    budget = g.uniform(0, 5000, size=(B, 1))
    shares = g.integers(0, 40, size=(B, 1)).astype(np.float64)
    return np.concatenate([p, budget, shares], 1).astype(np.float32)


def _server(eps=None, **kw):
    cfg = preset_config("flagship")
    if eps is not None:
        cfg.agent.epsilon = eps
    return PolicyServer(cfg, device=torch.device("cpu"), backend="torch", **kw)


def test_greedy_infer_matches_oracle_and_q():
    srv = _server()
    x = _rows(37)
    a, q = srv.infer(x, return_q=True)
    cfg = srv.cfg
    a_ref, q_ref = reference_select(srv.params, srv.layout, torch.from_numpy(x), history=201,
                                    feat_mode="relative", output_relu=False, budget0=cfg.env.budget,
                                    epsilon=cfg.agent.epsilon, ramp=cfg.agent.ramp, key_seed=srv.seed)
    assert torch.equal(a, a_ref) and torch.allclose(q, q_ref)
    assert a.dtype == torch.int32 and a.shape == (37,) and q.shape == (37, 3)
    assert torch.equal(a, q.argmax(1).to(torch.int32))


def test_epsilon_greedy_ramp_and_reproducible_draws():
    srv = _server()
    x = _rows(256, seed=1)
    greedy = srv.infer(x)
    # step 0: exploit probability min(eps, 0) = 0 -> every action is the random draw
    a0 = srv.infer(x, np.zeros(256))
    # step >> ramp: exploit with probability eps
    a_hi = srv.infer(x, np.full(256, 1e9))
    eps = srv.cfg.agent.epsilon
    agree = float((a_hi == greedy).float().mean())
    assert agree >= eps - 0.1
    # same seed, same batch sequence number -> the same draws
    srv2 = _server()
    srv2.seq = 1   # a0 was the server's second batch
    assert torch.equal(srv2.infer(x, np.zeros(256)), a0)
    assert not torch.equal(srv2.infer(x, np.zeros(256)), a0)   # the next batch draws anew
    assert set(a0.tolist()) <= {0, 1, 2} and len(set(a0.tolist())) == 3


def test_bad_rows_rejected():
    srv = _server()
    with pytest.raises(ValueError):
        srv.infer(np.zeros((2, 50), np.float32))
    with pytest.raises(ValueError):
        srv.infer(_rows(3), [1.0, 2.0])


def test_load_params_changes_the_policy():
    srv = _server()
    x = _rows(64, seed=2)
    a1, q1 = srv.infer(x, return_q=True)
    m = srv.cfg.model
    new = qn.init_params(srv.layout, m, seed=4321)
    srv.load_params(new)
    a2, q2 = srv.infer(x, return_q=True)
    assert not torch.allclose(q1, q2)
    with pytest.raises(ValueError):
        srv.load_params(torch.zeros(10))


def test_dynamic_batcher_groups_concurrent_requests():
    srv = _server()
    x = _rows(200, seed=3)
    want = srv.infer(x).tolist()
    out = [None] * 200
    with DynamicBatcher(srv, max_batch=64, max_delay_us=20000, greedy=True) as bat:
        def client(lo, hi):
            futs = [(i, bat.submit(x[i])) for i in range(lo, hi)]
            for i, f in futs:
                out[i] = f.result(timeout=30)

        ts = [threading.Thread(target=client, args=(k * 50, (k + 1) * 50)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        st = bat.stats()
    assert out == want
    assert st["requests"] == 200 and st["max_batch"] <= 64
    assert st["batches"] < 200   # requests were grouped
    with pytest.raises(RuntimeError):
        bat.submit(x[0])


def test_batcher_propagates_errors():
    srv = _server()
    with DynamicBatcher(srv, max_batch=8, max_delay_us=100) as bat:
        with pytest.raises(ValueError):
            bat.submit(np.zeros(7, np.float32))


@pytest.fixture
def system():
    s = ActorSystem("serve", loglevel="DEBUG")
    yield s
    s.terminate()


def test_serving_actor_answers_selection_action(system):
    kit = TestKit(system)
    srv = _server(eps=1.0)   # exploit probability min(1, step / ramp) = 1 at step 1e9: greedy
    x = _rows(5, seed=4)
    ref = srv.infer(x)
    act = system.actor_of(PolicyServingActor.props(srv))
    for i in range(5):
        kit.tell(act, P.SelectionAction(x[i:i + 1], 1e9))
    got = [kit.expect_msg_type(P.Action) for _ in range(5)]
    assert [g.index for g in got] == ref.tolist()
    assert srv.requests == 10 and srv.batches <= 6   # queued selections share launches


def test_serving_actor_wrong_shape_and_load_policy(system):
    kit = TestKit(system)
    srv = _server()
    act = system.actor_of(PolicyServingActor.props(srv))
    with EventFilter(system, IllegalArgumentException, occurrences=1).intercept():
        kit.tell(act, P.SelectionAction(list(range(10)), 0))
    new = qn.init_params(srv.layout, srv.cfg.model, seed=99)
    kit.tell(act, LoadPolicy(new))
    kit.expect_msg(PolicyLoaded)
    assert torch.equal(srv.params, new)


def test_http_front_end(tmp_path):
    from fastapi.testclient import TestClient

    from sharetrade.persist.checkpoint import CheckpointManager
    from sharetrade.serve.http import load_checkpoint_params, make_app

    srv = _server(eps=1.0)
    x = _rows(6, seed=8)
    with DynamicBatcher(srv, max_batch=16, max_delay_us=1000) as bat:
        c = TestClient(make_app(srv, bat, ckpt_root=str(tmp_path)))
        r = c.post("/select", json={"states": x.tolist(), "return_q": True})
        assert r.status_code == 200
        want = srv.infer(x).tolist()
        assert r.json()["actions"] == want and len(r.json()["q"]) == 6
        # the reference's message shape: greedy at step 1e9 with eps = 1
        r = c.post("/selection_action", json={"current_state": x[2].tolist(), "step": 1e9})
        assert r.status_code == 200 and r.json()["index"] == want[2]
        assert r.json()["action"] == ("Buy", "Sell", "Hold")[want[2]]
        assert c.post("/selection_action", json={"current_state": [1.0, 2.0], "step": 0}).status_code == 400
        assert c.post("/select", json={"states": [[1.0, 2.0]]}).status_code == 400
        # weights from an engine checkpoint (CheckpointManager directory)
        new = qn.init_params(srv.layout, srv.cfg.model, seed=77)
        CheckpointManager(str(tmp_path), interval=1).save(5, {"params": new, "step": torch.tensor([5])})
        assert torch.equal(load_checkpoint_params(str(tmp_path)), new)
        r = c.post("/load", json={"checkpoint": str(tmp_path)})
        assert r.status_code == 200 and torch.equal(srv.params, new)
        assert c.post("/load", json={"checkpoint": str(tmp_path / "missing")}).status_code == 400
        # only paths under the checkpoint root: absolute paths elsewhere and .. escapes are refused
        assert c.post("/load", json={"checkpoint": "/etc"}).status_code == 403
        assert c.post("/load", json={"checkpoint": "../"}).status_code == 403
        assert c.post("/load", json={"checkpoint": "."}).status_code == 200       # relative to the root
        assert TestClient(make_app(srv, bat)).post("/load", json={"checkpoint": str(tmp_path)}).status_code == 403
        h = c.get("/health").json()
        assert h["backend"] == "torch" and h["requests"] >= 8
        # binary route: float32 rows of state + step (step < 0: greedy), int8 actions back
        want = srv.infer(x).tolist()   # the weights loaded above
        body = np.concatenate([x, np.full((6, 1), -1.0, np.float32)], 1).astype("<f4").tobytes()
        r = c.post("/select_bin", content=body)
        assert r.status_code == 200 and [int(v) for v in np.frombuffer(r.content, np.int8)] == want
        one = np.concatenate([x[3], [1e9]]).astype("<f4").tobytes()
        r = c.post("/select_bin", content=one)   # one row: through the batcher (eps 1, step 1e9: greedy)
        assert r.status_code == 200 and int(np.frombuffer(r.content, np.int8)[0]) == want[3]
        one_greedy = np.concatenate([x[4], [-1.0]]).astype("<f4").tobytes()   # step < 0: greedy, not batched
        r = c.post("/select_bin", content=one_greedy)
        assert r.status_code == 200 and int(np.frombuffer(r.content, np.int8)[0]) == want[4]
        assert c.post("/select_bin", content=b"\x00" * 12).status_code == 400
        # mixed greedy / drawing rows in one body: the greedy rows stay greedy (eps 1 at step 1e9 = greedy
        # too; step 0 = always explore, so only the greedy rows are pinned)
        steps = np.array([-1.0, 0.0, -1.0, 1e9, 0.0, -1.0], np.float32)
        body = np.concatenate([x, steps[:, None]], 1).astype("<f4").tobytes()
        for _ in range(4):
            r = c.post("/select_bin", content=body)
            got = [int(v) for v in np.frombuffer(r.content, np.int8)]
            assert r.status_code == 200 and all(got[i] == want[i] for i in (0, 2, 3, 5)), (got, want)
        small = TestClient(make_app(srv, bat, max_bin_rows=2))
        assert small.post("/select_bin", content=body).status_code == 413
        m = c.get("/metrics").text
        assert 'sharetrade_serve_requests_total{route="select"} 6.0' in m
        assert 'sharetrade_serve_requests_total{route="select_bin"} 32.0' in m
        assert 'sharetrade_serve_requests_total{route="selection_action"} 1.0' in m
        assert 'sharetrade_serve_errors_total{route="selection_action"} 1.0' in m
        assert "sharetrade_serve_batch_rows_count 2.0" in m


def test_cli_serve_process():
    """``python -m sharetrade serve`` as a process: health and one SelectionAction over HTTP."""
    import os
    import socket
    import subprocess
    import sys
    import time

    import httpx

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    proc = subprocess.Popen([sys.executable, "-m", "sharetrade", "serve", "--device", "cpu", "--port", str(port)],
                            cwd=root, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        url = f"http://127.0.0.1:{port}"
        for _ in range(300):
            try:
                if httpx.get(url + "/health", timeout=1.0).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        else:
            raise AssertionError("server did not come up")
        r = httpx.post(url + "/selection_action", json={"current_state": _rows(1)[0].tolist(), "step": 5.0},
                       timeout=10.0)
        assert r.status_code == 200 and r.json()["action"] in ("Buy", "Sell", "Hold")
    finally:
        proc.terminate()
        proc.wait(timeout=30)


def test_serve_weights_from_engine_checkpoints(tmp_path):
    """Engine checkpoints in both layouts: a CheckpointManager directory and a sharded multi-rank one
    (newest committed step, rank 0; an uncommitted newer step is ignored)."""
    from sharetrade.parallel.dp_train import commit, save_shard
    from sharetrade.serve.http import load_checkpoint_params
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.envs_per_rank = 32
    eng = VectorEngine(cfg, device=torch.device("cpu"), envs=32, backend="torch")
    eng.run(2)
    save_shard(str(tmp_path), 2, 0, eng)
    commit(str(tmp_path), 2, 1)
    want = eng.params.clone()
    eng.run(1)
    save_shard(str(tmp_path), 3, 0, eng)   # not committed
    got = load_checkpoint_params(str(tmp_path))
    assert torch.equal(got, want)
    srv = _server()
    srv.load_params(got)
    x = _rows(4, seed=3)
    a_eng = PolicyServer(eng.cfg, params=want, device=torch.device("cpu"), backend="torch").infer(x)
    assert torch.equal(srv.infer(x), a_eng)


def test_engine_polyak_average_for_serving(tmp_path):
    """engine.ema_decay > 0: ema <- ema + (1 - d)(w - ema) after every update (host path here, the
    optimizer kernel on the GPU: tests/test_gpu_serve.py); checkpoints carry it and serving prefers it."""
    from sharetrade.persist.checkpoint import CheckpointManager
    from sharetrade.serve.http import load_checkpoint_params
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.ema_decay = 0.9
    eng = VectorEngine(cfg, device=torch.device("cpu"), envs=32, backend="torch")
    want = eng.params.clone()
    c = float(np.float32(1.0) - np.float32(0.9))
    for _ in range(3):
        eng.step()
        want = want + (eng.params - want) * c
    assert torch.equal(eng.params_ema, want) and not torch.equal(eng.params_ema, eng.params)
    assert eng.serving_params is eng.params_ema
    sd = eng.state_dict()
    assert torch.equal(sd["params_ema"], want)
    eng2 = VectorEngine(cfg, device=torch.device("cpu"), envs=32, backend="torch")
    eng2.load_state_dict(sd)
    assert torch.equal(eng2.params_ema, want)
    srv = PolicyServer.from_engine(eng, backend="torch")
    assert torch.equal(srv.params, want)
    assert torch.equal(PolicyServer.from_engine(eng, backend="torch", averaged=False).params, eng.params)
    CheckpointManager(str(tmp_path), interval=1).save(3, sd)
    assert torch.equal(load_checkpoint_params(str(tmp_path)), want)
    assert torch.equal(load_checkpoint_params(str(tmp_path), averaged=False), sd["params"])
    with pytest.raises(ValueError):
        cfg.engine.ema_decay = 1.0
        VectorEngine(cfg, device=torch.device("cpu"), envs=32, backend="torch")
