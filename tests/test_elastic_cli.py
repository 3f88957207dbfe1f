"""``python -m sharetrade engine --elastic N`` (CPU, gloo, 2 ranks): a rank that dies
(``SHARETRADE_FAIL_AT``) or hangs (``SHARETRADE_HANG_AT``: alive, heartbeat beating, no progress) mid-run
fails the generation; the launcher respawns it, every rank resumes from the newest committed shard, and
the job ends with final shards bit-identical to an uninterrupted run (the reference's backoff-supervised
worker replacement, `TrainerRouterActor.scala:46-58`, across processes)."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp, tag, env_extra=None, stall=60.0):
    d = os.path.join(tmp, tag)
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("SHARETRADE_FAIL_AT", None)
    env.pop("SHARETRADE_HANG_AT", None)
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "sharetrade", "engine", "--preset", "intended", "--device", "cpu",
           "--dist-backend", "gloo", "--elastic", "2", "--steps", "12", "--envs", "4", "--ckpt-dir",
           os.path.join(d, "ckpt"), "--ckpt-every", "4", "--final-dir", os.path.join(d, "final"), "--log-every", "0",
           "--stall-timeout", str(stall), "--set", "data.source=random_walk", "--set", "data.length=260",
           "--set", "model.hidden=[32]"]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    from sharetrade.persist import checkpoint as ck

    finals = [ck.load(os.path.join(d, "final", f"final-rank-{r}.stck"))[0] for r in range(2)]
    return res, finals


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    return _run(str(tmp_path_factory.mktemp("ref")), "ref")


def _same(a, b):
    for x, y in zip(a, b):
        assert torch.equal(x["params"], y["params"])
        for k in ("env_pos", "env_budget", "env_shares", "opt_s1", "opt_s2", "step"):
            assert torch.equal(x[k], y[k]), k


def test_clean_elastic_run(reference):
    res, finals = reference
    assert res["ok"] and res["restarts"] == 0
    assert int(finals[0]["step"][0]) == 12
    assert torch.equal(finals[0]["params"], finals[1]["params"])      # one learner, two ranks


def test_rank_death_recovers_bit_exactly(reference, tmp_path):
    res, finals = _run(str(tmp_path), "fail", {"SHARETRADE_FAIL_AT": "1:6:0"})
    assert res["ok"] and res["restarts"] == 1, res
    assert res["generations"][0]["exitcodes"]["1"] == 17
    _same(reference[1], finals)


def test_hung_rank_detected_and_recovered(reference, tmp_path):
    res, finals = _run(str(tmp_path), "hang", {"SHARETRADE_HANG_AT": "0:6:0"}, stall=6.0)
    assert res["ok"] and res["restarts"] == 1, res
    assert res["flagged"]                                         # the watchdog flagged the stalled generation
    _same(reference[1], finals)
