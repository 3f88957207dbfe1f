"""Multi-process data parallelism on CPU (gloo): the same code path the MI355X
node runs over RCCL, world_size 2 and 4.

Sync-DP equivalence: N ranks holding E envs each must produce exactly the
parameters of one process holding all N*E envs (global env ids index the RNG,
the loss is pre-scaled by the global batch, gradients are all-reduced)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(opt="adam"):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship")
    cfg.engine.dtype = "fp32"
    cfg.agent.optimizer = opt
    cfg.agent.epsilon = 0.6
    cfg.agent.ramp = 5.0
    cfg.model.hidden = [32, 32]
    return cfg


def _prices(n, T=260):
    from sharetrade.data.prices import random_walk

    return torch.from_numpy(random_walk(T, 50.0, 0.02, 11, n_series=n).astype(np.float32))


def _worker(rank, world, port, E, steps, out_dir, opt, compress):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from sharetrade.parallel import dist as D
    from sharetrade.trainer.engine import VectorEngine

    ctx = D.init(backend="gloo", device="cpu")
    cfg = _cfg(opt)
    cfg.engine.grad_compress = compress
    cfg.engine.bucket_mb = 0.01 if compress == "" else 4.0   # force several buckets in the fp32 case
    bank = _prices(E * world)[rank * E:(rank + 1) * E]
    eng = VectorEngine(cfg, prices=bank, device=torch.device("cpu"), rank=rank, world_size=world, group=ctx.group,
                       envs=E, backend="torch")
    if rank != 0:
        eng.params.add_(1.0)          # broadcast must overwrite this
    eng.sync_params_from(0)
    eng.run(steps)
    summ = D.global_mean_std(ctx, eng.current_portfolios())
    gathered = D.all_gather_values(ctx, eng.current_portfolios())
    torch.save({"params": eng.params, "summary": summ, "gathered": gathered,
                "done": D.all_done(ctx, True)}, os.path.join(out_dir, f"r{rank}.pt"))
    D.shutdown(ctx)


def _run_dp(world, E, steps, opt="adam", compress=""):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, port, E, steps, d, opt, compress), nprocs=world, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_sync_dp_equals_single_process(world):
    from sharetrade.trainer.engine import VectorEngine

    E, steps = 3, 6
    res = _run_dp(world, E, steps)
    for r in res[1:]:
        assert torch.equal(r["params"], res[0]["params"])        # replicas stay identical
    single = VectorEngine(_cfg(), prices=_prices(E * world), device=torch.device("cpu"), envs=E * world,
                          backend="torch")
    single.run(steps)
    rel = float((res[0]["params"] - single.params).norm() / single.params.norm())
    assert rel < 1e-5, rel
    # cross-rank aggregation == single-process aggregation
    pf = single.current_portfolios().double()
    s = res[0]["summary"]
    assert s["n"] == E * world
    assert abs(s["mean"] - float(pf.mean())) < 1e-6 * abs(float(pf.mean()))
    assert torch.allclose(res[0]["gathered"].double(), pf, rtol=1e-6)
    assert res[0]["done"] is True


def test_dp_bf16_wire_compression_stays_close():
    res = _run_dp(2, 3, 4, opt="sgd", compress="bf16")
    assert torch.equal(res[0]["params"], res[1]["params"])
    res32 = _run_dp(2, 3, 4, opt="sgd", compress="")
    rel = float((res[0]["params"] - res32[0]["params"]).norm() / res32[0]["params"].norm())
    assert rel < 1e-2


def _timing_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from sharetrade.parallel import dist as D

    ctx = D.init(backend="gloo", device="cpu")
    gs = D.GradSync(ctx, 1000)
    g = torch.full((1000,), float(rank + 1))
    assert gs.pop_timing_ms() is None
    gs.enable_timing()
    for _ in range(3):
        gs.all_reduce(g)
    ms = gs.pop_timing_ms()
    torch.save({"ms": ms, "g0": float(g[0]), "calls": gs.calls, "again": gs.pop_timing_ms()},
               os.path.join(out_dir, f"t{rank}.pt"))
    D.shutdown(ctx)


def test_grad_sync_records_allreduce_time():
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_timing_worker, args=(2, port, d), nprocs=2, join=True, start_method="spawn")
        res = [torch.load(os.path.join(d, f"t{r}.pt"), weights_only=True) for r in range(2)]
    for r in res:
        assert r["ms"] is not None and r["ms"] >= 0.0 and r["again"] is None
        assert r["calls"] == 3 and r["g0"] == 3.0 * 2 ** 2   # 1 + 2, then doubled by each further in-place sum


def _torchrun(args, nproc=2):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "sharetrade", "engine",
           "--preset", "intended", "--device", "cpu", "--envs", "3", "--log-every", "0",
           "--set", "data.source=random_walk", "--set", "data.length=300"] + args
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=root, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


def test_cli_engine_sharded_checkpoint_resume_two_ranks(tmp_path):
    """``python -m sharetrade engine`` under torchrun: every rank writes its own shard, rank 0
    commits; ``--resume`` loads each rank's own shard.  3 steps + resume 3 steps must write
    the same step-6 shards (byte-identical, deterministic writer) as 6 uninterrupted steps."""
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _torchrun(["--steps", "6", "--ckpt-dir", a, "--ckpt-every", "3"])
    _torchrun(["--steps", "3", "--ckpt-dir", b, "--ckpt-every", "3"])
    assert sorted(os.listdir(b)) == ["step-000000003"]
    assert sorted(os.listdir(os.path.join(b, "step-000000003"))) == ["COMMIT", "rank-0.stck", "rank-1.stck"]
    _torchrun(["--steps", "3", "--ckpt-dir", b, "--ckpt-every", "3", "--resume"])
    for r in range(2):
        pa = os.path.join(a, "step-000000006", f"rank-{r}.stck")
        pb = os.path.join(b, "step-000000006", f"rank-{r}.stck")
        assert open(pa, "rb").read() == open(pb, "rb").read(), f"rank {r} diverged after resume"
    from sharetrade.persist import checkpoint as ck

    s0, _ = ck.load(os.path.join(a, "step-000000006", "rank-0.stck"))
    s1, _ = ck.load(os.path.join(a, "step-000000006", "rank-1.stck"))
    assert torch.equal(s0["params"], s1["params"])                 # sync DP: one learner
    assert not torch.equal(s0["env_budget"], s1["env_budget"])     # each rank owns its own envs
    assert int(s0["opt_t"][0]) == 6
