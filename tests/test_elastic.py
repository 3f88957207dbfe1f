"""Elastic recovery (CPU, gloo): a rank dies mid-run, the generation is respawned,
resumes from the last committed sharded checkpoint and finishes bit-identically to
an uninterrupted run (the cross-process analogue of the router replacing a dead
worker and re-sending Train)."""
import os
import tempfile

import pytest
import torch

from sharetrade.config import preset_config
from sharetrade.parallel.dp_train import dp_worker
from sharetrade.parallel.elastic import ElasticRunner, Heartbeat, Watchdog
from sharetrade.persist import checkpoint as ck


def _cfg():
    cfg = preset_config("flagship")
    cfg.engine.dtype = "fp32"
    cfg.model.hidden = [32, 32]
    cfg.agent.epsilon = 0.6
    cfg.agent.ramp = 5.0
    return cfg.to_dict()


def _run(world, steps, fail_at=None, ckpt_every=3):
    d = tempfile.mkdtemp()
    env = {"SHARETRADE_FAIL_AT": fail_at} if fail_at else {}
    r = ElasticRunner(dp_worker, world, args=(_cfg(), steps, os.path.join(d, "ckpt"), ckpt_every, 3,
                                              os.path.join(d, "out")), max_restarts=2, env=env).run()
    finals = [ck.load(os.path.join(d, "out", f"final-rank-{k}.stck"))[0] for k in range(world)] if r.ok else None
    return r, finals


def test_failure_is_recovered_bit_exactly():
    ref, ref_f = _run(2, 8)
    assert ref.ok and ref.restarts == 0
    got, got_f = _run(2, 8, fail_at="1:5")          # rank 1 dies before step 5 of generation 0
    assert got.ok and got.restarts == 1
    assert got.generations[0].exitcodes[1] == 17     # the injected failure was observed
    for a, b in zip(ref_f, got_f):
        assert torch.equal(a["params"], b["params"])
        assert torch.equal(a["env_budget"], b["env_budget"])
        assert torch.equal(a["env_pos"], b["env_pos"])
        assert int(a["step"][0]) == int(b["step"][0]) == 8


def test_gives_up_after_max_restarts():
    d = tempfile.mkdtemp()
    # fails in every generation it reaches: gen 0 at step 1; gens 1, 2 never checkpointed past 0
    env = {"SHARETRADE_FAIL_AT": "0:1"}
    r = ElasticRunner(dp_worker, 2, args=(_cfg(), 4, os.path.join(d, "c"), 0, 2, os.path.join(d, "o")),
                      max_restarts=0, env=env).run()
    assert not r.ok and len(r.generations) == 1


def test_heartbeat_watchdog_flags_stale_rank():
    store = torch.distributed.HashStore()
    hb0 = Heartbeat(store, 0, interval_s=0.05).start()
    Heartbeat(store, 1, interval_s=0.05).beat()         # rank 1 beats once, then "dies"
    dead = []
    wd = Watchdog(store, 2, timeout_s=0.3, on_dead=dead.append, poll_s=0.05).start()
    import time

    time.sleep(0.8)
    wd.stop()
    hb0.stop()
    assert dead == [1]


def test_hung_rank_is_detected_by_watchdog_and_recovered():
    """A rank that hangs (alive, heartbeat thread beating, main loop stuck) is flagged by the
    launcher's progress watchdog within seconds -- not the generation timeout -- and the
    respawned generation finishes bit-identically to an uninterrupted run."""
    import time

    ref, ref_f = _run(2, 8)
    d = tempfile.mkdtemp()
    t0 = time.monotonic()
    r = ElasticRunner(dp_worker, 2, args=(_cfg(), 8, os.path.join(d, "ckpt"), 3, 3, os.path.join(d, "out")),
                      max_restarts=2, env={"SHARETRADE_HANG_AT": "0:4"}, stall_timeout_s=3.0,
                      gen_timeout_s=300.0).run()
    assert r.ok and r.restarts == 1
    assert (0, 0) in r.flagged or (0, 1) in r.flagged   # rank 0 hung; rank 1 blocks in its collective
    assert time.monotonic() - t0 < 120
    got_f = [ck.load(os.path.join(d, "out", f"final-rank-{k}.stck"))[0] for k in range(2)]
    for a, b in zip(ref_f, got_f):
        assert torch.equal(a["params"], b["params"])
        assert torch.equal(a["env_pos"], b["env_pos"])


def test_watchdog_flags_stalled_progress():
    import time

    store = torch.distributed.HashStore()
    hb = Heartbeat(store, 0, interval_s=0.05).start()    # alive ...
    hb.progress(3)                                        # ... but never advances past step 3
    wd = Watchdog(store, 1, timeout_s=5.0, poll_s=0.05, stall_timeout_s=0.3).start()
    time.sleep(0.8)
    wd.stop()
    hb.stop()
    assert wd.dead == [0]


def test_watchdog_ignores_cleanly_finished_rank():
    """A rank that exited 0 stops beating by design; the watchdog must not flag it (a finished
    generation would otherwise be failed and restarted)."""
    import time

    store = torch.distributed.HashStore()
    hb0 = Heartbeat(store, 0, interval_s=0.05).start()
    Heartbeat(store, 1, interval_s=0.05).beat()          # rank 1 beat, then exited with code 0
    wd = Watchdog(store, 2, timeout_s=0.3, poll_s=0.05)
    wd.finished.add(1)
    wd.start()
    time.sleep(0.8)
    wd.stop()
    hb0.stop()
    assert wd.dead == []
