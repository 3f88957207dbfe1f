"""Data parallelism of the config-4 / config-5 learners (sharetrade/trainer/runs.py ``ctx=``):

* two ranks sharing cuda:0 over gloo (the box has one GPU; the 8-GPU run uses RCCL) run their own envs
  and replay, start from rank 0's parameters and sum gradients before every Adam step -- after a few
  captured iterations both ranks hold bit-identical parameters while their env state differs;
* over a one-rank RCCL group with world_size forced to 2, both captured DP forms -- the all-reduce
  between two graphs (gradients | Adam), and the all-reduce inside the update graph (config 4: per
  layer on a comm stream beside the backward) -- match the eager DP iteration (counters and env state
  exact, weights up to fp32 reduction order)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

_DEEP = dict(envs=256, batch=256, replay_capacity=4096, hidden=[256, 256], overlap_act=True, target_every=3)
_REC = dict(envs=256, seq=8, batch=128, bars=600, ep_len=5, replay_segments=2048, burn_in=1, overlap_act=True,
            target_every=3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(kind):
    from sharetrade.config import preset_config

    return preset_config("flagship" if kind == "deep" else "recurrent")


def _params(kind, st):
    if kind == "recurrent":
        return st["flat"]
    return torch.cat([st[f"{n}{l}"].flatten() for l in range(3) for n in ("W", "b", "Wt", "bt")])


def _gloo_worker(rank, world, port, kind, iters, out, ckpt_every=None, resume=False, eps0=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sharetrade.parallel.dist import DistContext
    from sharetrade.trainer.runs import run

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext(rank, world, 0, "gloo", dev, dist.group.WORLD)
    kw = dict(_DEEP if kind == "deep" else _REC)
    cfg = _cfg(kind)
    if eps0:
        cfg.agent.epsilon = 0.0      # actions from the Philox draws only: trajectories do not depend on Q
    res = run(kind, cfg, iters, device=dev, ctx=ctx, ckpt_dir=out, ckpt_every=ckpt_every or iters,
              resume=resume, log_every=0, **kw)
    assert res["world_size"] == world and res["iterations"] == iters
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["deep", "recurrent"])
def test_two_rank_dp_keeps_parameters_identical(native_built, kind):
    from sharetrade.persist.checkpoint import CheckpointManager, load
    from sharetrade.trainer.runs import build

    iters, world = 7, 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gloo_worker, args=(world, _port(), kind, iters, d), nprocs=world, join=True,
                           start_method="spawn")
        st = [load(CheckpointManager(os.path.join(d, f"rank{r}")).latest())[0] for r in range(world)]
    p0, p1 = _params(kind, st[0]), _params(kind, st[1])
    assert torch.isfinite(p0).all()
    assert torch.equal(p0, p1)                       # one shared model
    env_key = "pos" if kind == "recurrent" else "budget"
    assert not torch.equal(st[0][env_key], st[1][env_key])      # each rank its own envs
    # and the model trained away from rank 0's initial parameters
    fresh = build(kind, _cfg(kind), torch.device("cuda", 0), **dict(_DEEP if kind == "deep" else _REC))
    assert not torch.equal(_params(kind, {k: v.cpu() for k, v in fresh.state_dict().items()}), p0)


@pytest.mark.parametrize("kind", ["deep", "recurrent"])
def test_two_rank_dp_resume_continues_the_run(native_built, kind):
    """Per-rank checkpoints: a 2-rank run stopped after iteration 4 and resumed to 7 ends where the
    uninterrupted 7-iteration run ends (env state / counters exact, weights up to fp32 reduction order)."""
    import shutil

    from sharetrade.persist.checkpoint import CheckpointManager, load

    world = 2
    with tempfile.TemporaryDirectory() as d:
        a, b = os.path.join(d, "a"), os.path.join(d, "b")
        mp.start_processes(_gloo_worker, args=(world, _port(), kind, 7, a, 7, False, True), nprocs=world, join=True,
                           start_method="spawn")
        mp.start_processes(_gloo_worker, args=(world, _port(), kind, 4, b, 4, False, True), nprocs=world, join=True,
                           start_method="spawn")
        for r in range(world):     # keep only the iteration-4 checkpoints, then resume to 7
            mgr = CheckpointManager(os.path.join(b, f"rank{r}"))
            assert [os.path.basename(p) for p in mgr.list()] == ["ckpt-000000000004.stck"]
        mp.start_processes(_gloo_worker, args=(world, _port(), kind, 7, b, 7, True, True), nprocs=world, join=True,
                           start_method="spawn")
        for r in range(world):
            sa = load(CheckpointManager(os.path.join(a, f"rank{r}")).latest())[0]
            sb = load(CheckpointManager(os.path.join(b, f"rank{r}")).latest())[0]
            assert torch.equal(sa["counters"], sb["counters"])
            env_keys = ("pos", "ep_start", "rctrl", "position") if kind == "recurrent" else \
                ("rp_ctrl", "env_ctrl", "t_ctr", "budget", "shares")
            for k in env_keys:
                assert torch.equal(sa[k], sb[k]), (r, k)
            pa, pb = _params(kind, sa).float(), _params(kind, sb).float()
            assert torch.allclose(pa, pb, rtol=1e-3, atol=1e-5), (r, float((pa - pb).abs().max()))
        shutil.rmtree(d, ignore_errors=True)


def _rccl_worker(_rank, port, kind, fast, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sharetrade.parallel.dist import DistContext
    from sharetrade.trainer.runs import build, run

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ctx = DistContext(0, 2, 0, "nccl", dev, dist.group.WORLD)     # the DP code path over one rank
    cfg = _cfg(kind)
    cfg.agent.epsilon = 0.0
    kw = dict(_DEEP if kind == "deep" else _REC, world_size=2)
    if kind == "deep" and not fast:
        # bit-reproducible weight gradients (no split-K atomics), as in tests/test_gpu_runs.py
        kw.update(dw_gemm="hip", concurrent=False, batched_fwd=False, dual_bwd=False)
    res = {}
    # eager; captured with the all-reduce between two graphs; captured with the all-reduce inside the
    # update graph (config 4: per layer on a comm stream)
    for mode, graph, cap in (("eager", False, True), ("split", True, False), ("ingraph", True, True)):
        d = build(kind, cfg, dev, **kw)
        run(kind, cfg, 6, device=dev, ctx=ctx, learner=d, graph=graph, capture_sync=cap, log_every=0)
        if graph:
            assert (d._g_pre_act is not None) == (not cap) and (d._g_iter is not None) == cap
            assert (getattr(d, "layer_sync", None) is not None) == (cap and kind == "deep")
        torch.cuda.synchronize()
        res[mode] = d.state_dict()
    torch.save(res, os.path.join(out, "cap.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,fast", [("deep", False), ("deep", True), ("recurrent", True)])
def test_dp_capture_matches_eager_over_rccl(native_built, kind, fast):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rccl_worker, args=(_port(), kind, fast, d), nprocs=1, join=True, start_method="spawn")
        res = torch.load(os.path.join(d, "cap.pt"), weights_only=True)
    # as tests/test_gpu_runs.py: weight-dependent values equal up to fp32 reduction order (float
    # atomics), env / replay / counters exact (epsilon = 0: actions do not depend on Q)
    approx = ("flat", "mflat", "vflat", "tflat", "h", "rh0", "loss", "stats") if kind == "recurrent" \
        else ("loss", "stats")
    e = res["eager"]
    for mode in ("split", "ingraph"):
        g = res[mode]
        assert e.keys() == g.keys() and torch.equal(e["counters"], g["counters"])
        for k in e:
            x, y = e[k], g[k]
            if k in approx or (kind == "deep" and k.rstrip("0123456789") in ("W", "b", "Wm", "Wv", "bm", "bv", "Wt",
                                                                              "bt")):
                assert torch.allclose(x.float(), y.float(), rtol=1e-4, atol=1e-5), (mode, k)
            elif x.is_floating_point():
                assert torch.equal(x.float().nan_to_num(-7.0), y.float().nan_to_num(-7.0)), (mode, k)
            else:
                assert torch.equal(x, y), (mode, k)
