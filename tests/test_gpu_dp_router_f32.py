"""The router fan-out (DP plane) on GPU fp32 ranks: two rank processes sharing cuda:0 (gloo collectives on
device tensors), each running the batched fp32 MFMA step (csrc/mlp_f32_mfma.hip, 1,024 envs per rank).  At
world_size > 1 the step runs deterministic (engine.f32_deterministic='auto': split-K partials and bias
column-sum partials added in a fixed order, no fp32 atomics), so a rank killed mid-episode and resumed from the
last committed shard ends with bit-identical parameters to a run without the failure -- the property
tests/test_dp_router.py pins on the CPU torch backend (`TrainerRouterActor.scala:116-120,141-146`).
"""
import os

import pytest

from test_dp_router import _cfg

pytestmark = pytest.mark.gpu


def _run(world, fail=None, tmp=None, envs=1024):
    from sharetrade.app import run

    old = os.environ.pop("SHARETRADE_FAIL_AT", None)
    if fail:
        os.environ["SHARETRADE_FAIL_AT"] = fail
    try:
        cfg = _cfg("intended")
        cfg.engine.dtype = "fp32"
        return run(cfg, engine="vector", device="cpu", max_prices=240, quiet=True, gpus=world,
                   dp=dict(device="cuda", backend="gloo", same_device=True, envs_per_rank=envs, ckpt_every=8,
                           ckpt_dir=str(tmp) if tmp else None,
                           group_kw=dict(stall_timeout_s=90.0, pg_timeout_s=60.0)))
    finally:
        os.environ.pop("SHARETRADE_FAIL_AT", None)
        if old is not None:
            os.environ["SHARETRADE_FAIL_AT"] = old


def test_gpu_fp32_rank_death_recovers_bit_exactly(tmp_path):
    ref = _run(2, tmp=tmp_path / "ref")
    got = _run(2, fail="1:20:0", tmp=tmp_path / "fail")
    assert ref["completed"] == 1.0 and got["completed"] == 1.0, (ref, got)
    assert ref["dp"]["deaths"] == []
    assert [d[:2] for d in got["dp"]["deaths"]] == [(0, 1)]
    assert all(r["start"] == 16 for r in got["dp"]["ranks"])
    crc_ref = [r["params_crc"] for r in ref["dp"]["ranks"]]
    crc_got = [r["params_crc"] for r in got["dp"]["ranks"]]
    print(f"[meas] fp32 GPU ranks params_crc ref={crc_ref} recovered={crc_got}")
    assert len(set(crc_ref)) == 1
    assert crc_got == crc_ref
    assert got["avg"] == ref["avg"] and got["std"] == ref["std"]
