"""The router fan-out as the data-parallel plane (CPU, gloo): ``run(engine="vector", gpus=N)``.

Every routee of the ``TrainerRouterActor`` is backed by one rank process of a torch.distributed group
(`sharetrade/trainer/dp_actors.py`, `sharetrade/parallel/rankgroup.py`).  ``StartTraining`` broadcasts
``Train`` (`TrainerRouterActor.scala:86-88`), the ranks run one synchronous-DP episode, ``GetAvg`` /
``GetStd`` are the ranks' all-env reduction, and a rank killed mid-episode (``SHARETRADE_FAIL_AT``) is
replaced: its routee is stopped, the router creates a new one and re-sends ``Train``
(`TrainerRouterActor.scala:101-102,116-120,141-146`), the group respawns and resumes from the last
committed shard -- and ends with exactly the parameters of a run without the failure.
"""
import os

import pytest

from sharetrade.config import preset_config


def _cfg(preset="test"):
    cfg = preset_config(preset)
    cfg.persist.journal_plugin = "inmemory"
    cfg.router.poll_interval_s = 0.2
    cfg.env.progress_every = 0
    return cfg


def _run(world, fail=None, preset="test", prices=240, envs=3, ckpt_every=8, tmp=None):
    from sharetrade.app import run

    old = os.environ.pop("SHARETRADE_FAIL_AT", None)
    if fail:
        os.environ["SHARETRADE_FAIL_AT"] = fail
    try:
        return run(_cfg(preset), engine="vector", device="cpu", max_prices=prices, quiet=True, gpus=world,
                   dp=dict(device="cpu", backend="gloo", envs_per_rank=envs, ckpt_every=ckpt_every,
                           ckpt_dir=str(tmp) if tmp else None,
                           group_kw=dict(stall_timeout_s=60.0, pg_timeout_s=30.0)))
    finally:
        os.environ.pop("SHARETRADE_FAIL_AT", None)
        if old is not None:
            os.environ["SHARETRADE_FAIL_AT"] = old


def test_two_ranks_reference_semantics(tmp_path):
    """reference_compat semantics on 2 ranks: every worker ends at its budget -> 2400.0 / 0.0, over all envs."""
    res = _run(2, tmp=tmp_path)
    assert res["completed"] == 1.0, res
    assert res["avg"] == 2400.0 and res["std"] == 0.0
    dp = res["dp"]
    assert dp["world"] == 2 and dp["deaths"] == [] and dp["generation"] == 0
    assert dp["global"]["n"] == 2 * 3                       # every env of both ranks
    assert len({r["params_crc"] for r in dp["ranks"]}) == 1   # the ranks hold identical parameters


@pytest.mark.parametrize("world", [2, 4])
def test_rank_death_is_replaced_and_resumed(world, tmp_path):
    """A rank dies at step 20 of the first generation: its routee is replaced and re-sent Train, the
    group respawns from the step-16 commit, and the episode ends with the parameters of a clean run."""
    ref = _run(world, preset="intended", tmp=tmp_path / "ref")
    got = _run(world, fail="1:20:0", preset="intended", tmp=tmp_path / "fail")
    assert ref["completed"] == 1.0 and got["completed"] == 1.0, (ref, got)
    assert ref["dp"]["deaths"] == []
    assert [d[:2] for d in got["dp"]["deaths"]] == [(0, 1)]          # generation 0, rank 1
    assert got["dp"]["generation"] == 1
    assert all(r["start"] == 16 for r in got["dp"]["ranks"])          # resumed from the last commit
    assert [r["params_crc"] for r in got["dp"]["ranks"]] == [r["params_crc"] for r in ref["dp"]["ranks"]]
    assert got["avg"] == ref["avg"] and got["std"] == ref["std"]
