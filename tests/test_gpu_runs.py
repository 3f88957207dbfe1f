"""Training runs of the config-4 / config-5 learners (sharetrade/trainer/runs.py): checkpoint after
iteration k, resume in a fresh learner, continue -- the same env trajectories, replay contents and
counters as the uninterrupted run, parameters within fp32 reduction-order noise."""
import os
import shutil
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _deep(cfg):
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer.deep import DeepDQN

    prices = torch.from_numpy(random_walk(400, 50.0, 0.02, 4, n_series=256).astype(np.float32))
    # hipBLASLt weight gradients, no split-K forward / dual launches: a run that is bit-reproducible
    return DeepDQN(cfg, torch.device("cuda", 0), envs=256, batch=256, replay_capacity=4096, prices=prices,
                   dw_gemm="hip", concurrent=False, batched_fwd=False, dual_bwd=False, overlap_act=True,
                   target_every=4)


def _rec(cfg):
    from sharetrade.trainer.recurrent import RecurrentDQN

    return RecurrentDQN(cfg, torch.device("cuda", 0), envs=256, seq=8, batch=128, bars=600, ep_len=5,
                        replay_segments=2048, burn_in=1, overlap_act=True, target_every=4)


def _cfg(kind):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship" if kind == "deep" else "recurrent")
    if kind == "deep":
        cfg.model.hidden = [256, 256]
    cfg.agent.epsilon = 0.0      # every action is a Philox draw: trajectories do not depend on Q
    return cfg


@pytest.mark.parametrize("kind", ["deep", "recurrent"])
def test_resume_continues_the_uninterrupted_run(native_built, kind):
    from sharetrade.persist.checkpoint import CheckpointManager
    from sharetrade.trainer.runs import run

    make = _deep if kind == "deep" else _rec
    d = tempfile.mkdtemp()
    try:
        a = make(_cfg(kind))
        ra = run(kind, _cfg(kind), 7, ckpt_dir=os.path.join(d, "a"), ckpt_every=3, log_every=0, learner=a,
                 metrics_path=os.path.join(d, "m.jsonl"))
        assert ra["iterations"] == 7 and a.updates == 7
        mgr = CheckpointManager(os.path.join(d, "a"))
        assert [os.path.basename(p) for p in mgr.list()] == ["ckpt-000000000003.stck", "ckpt-000000000006.stck"]
        os.makedirs(os.path.join(d, "b"))
        shutil.copy(os.path.join(d, "a", "ckpt-000000000003.stck"), os.path.join(d, "b"))
        b = make(_cfg(kind))
        rb = run(kind, _cfg(kind), 7, ckpt_dir=os.path.join(d, "b"), resume=True, log_every=0, learner=b)
        assert rb["iterations"] == 7 and b.updates == 7
        sa, sb = a.state_dict(), b.state_dict()
        assert sa.keys() == sb.keys()
        # weight-dependent values: equal up to fp32 reduction order; env / replay / counters: exact
        # (stats: float sums accumulated with atomics from many workgroups -- order-dependent bits)
        approx = ("flat", "mflat", "vflat", "tflat", "h", "rh0", "loss", "stats") if kind == "recurrent" \
            else ("loss", "stats")
        for k in sa:
            x, y = sa[k], sb[k]
            weighty = k in approx or (kind == "deep" and k.rstrip("0123456789") in ("W", "b", "Wm", "Wv", "bm", "bv",
                                                                                   "Wt", "bt"))
            if weighty:
                assert torch.allclose(x.float(), y.float(), rtol=1e-4, atol=1e-5), k
            elif x.is_floating_point():
                assert torch.equal(x.float().nan_to_num(-7.0), y.float().nan_to_num(-7.0)), k
            else:
                assert torch.equal(x, y), k
    finally:
        shutil.rmtree(d, ignore_errors=True)
