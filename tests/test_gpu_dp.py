"""Data parallelism through the native HIP step on the GPU (2 ranks sharing cuda:0 over
gloo — the same engine code the 8-GPU RCCL run executes; the box has one GPU)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(kernel):
    from sharetrade.config import preset_config

    cfg = preset_config("flagship")
    cfg.agent.optimizer = "sgd"
    cfg.agent.lr = 1e-2
    if kernel == "fp32":
        cfg.engine.dtype = "fp32"
    if kernel == "bf16_knobs":   # the ws knob build + target pass (agent.target_every / double_dqn)
        cfg.agent.target_every, cfg.agent.double_dqn, cfg.agent.reward_scale = 2, True, 2.0
    return cfg


def _bank(n, T=400):
    from sharetrade.data.prices import random_walk

    return torch.from_numpy(random_walk(T, 50.0, 0.02, 3, n_series=n).astype(np.float32))


def _worker(rank, world, port, E, steps, kernel, out, overlap=False, evaluate=False, graph=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    cfg = _cfg(kernel)
    cfg.engine.dp_overlap = overlap
    eng = VectorEngine(cfg, prices=_bank(E * world)[rank * E:(rank + 1) * E], device=dev, rank=rank,
                       world_size=world, group=dist.group.WORLD, envs=E)
    assert eng.backend == "native"
    eng.sync_params_from(0)
    res = {}
    if graph:
        # gloo: the sync-DP step as two captured graphs around the host-side all-reduce
        res["captured"] = eng.capture_graph(warmup=0)
    eng.run(steps)
    if evaluate:
        # a frozen-weight greedy episode in the middle of (overlapped) training: the parameters and the
        # pending gradient of the last training step survive it (greedy_episode_returns raises if the
        # evaluation moved the weights)
        eng.flush_pending()          # (the last training step's delayed update, applied before the snapshot)
        before = eng.params.detach().clone()
        res["greedy"] = benchkit.greedy_episode_returns(eng, world, dist.group.WORLD)["mean"]
        assert torch.equal(eng.params, before)
        eng.run(2)
    eng.flush_pending()
    torch.cuda.synchronize()
    res.update({"params": eng.params.cpu(), "budget": eng.state.budget.cpu()})
    if eng.params_target is not None:
        res["target"] = eng.params_target.cpu()
    torch.save(res, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kernel", ["bf16", "fp32", "bf16_knobs"])
def test_native_dp_two_ranks_match_single_process(native_built, kernel):
    from sharetrade.trainer.engine import VectorEngine

    E, steps, world = 64, 4, 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _port(), E, steps, kernel, d), nprocs=world, join=True,
                           start_method="spawn")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["params"], res[1]["params"])
    single = VectorEngine(_cfg(kernel), prices=_bank(E * world), device=torch.device("cuda", 0), envs=E * world)
    single.run(steps)
    torch.cuda.synchronize()
    p = single.params.cpu()
    rel = float((res[0]["params"] - p).norm() / p.norm())
    assert rel < (1e-5 if kernel == "fp32" else 1e-3), rel
    assert torch.equal(torch.cat([res[0]["budget"], res[1]["budget"]]), single.state.budget.cpu())


def test_overlapped_dp_is_rank_consistent_and_one_step_delayed(native_built):
    """dp_overlap: every rank applies the same (one-step delayed) gradients; the trajectory stays
    close to strict sync DP and the first step is identical (same initial weights)."""
    E, steps, world = 64, 6, 2
    out = {}
    for ov in (False, True):
        with tempfile.TemporaryDirectory() as d:
            mp.start_processes(_worker, args=(world, _port(), E, steps, "bf16", d, ov), nprocs=world, join=True,
                               start_method="spawn")
            out[ov] = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    a, b = out[True]
    assert torch.equal(a["params"], b["params"]) and torch.isfinite(a["params"]).all()
    p_sync = out[False][0]["params"]
    rel = float((a["params"] - p_sync).norm() / p_sync.norm())
    assert 0.0 < rel < 5e-2, rel


def test_overlapped_dp_with_target_net_is_rank_consistent(native_built):
    """dp_overlap + the target net / Double DQN on the ws kernel: the target copy follows the delayed update
    on every rank, so both ranks end with identical parameters."""
    E, world = 64, 2
    for steps in (7, 6):
        with tempfile.TemporaryDirectory() as d:
            mp.start_processes(_worker, args=(world, _port(), E, steps, "bf16_knobs", d, True), nprocs=world,
                               join=True, start_method="spawn")
            res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
        assert torch.equal(res[0]["params"], res[1]["params"]) and torch.isfinite(res[0]["params"]).all()
        assert torch.equal(res[0]["target"], res[1]["target"])
        if steps % 2 == 0:
            # the last step is a target boundary (target_every = 2): after flush_pending the target holds the
            # fully updated parameters, as in synchronous training
            assert torch.equal(res[0]["target"], res[0]["params"])
        else:
            assert not torch.equal(res[0]["target"], res[0]["params"])


def test_overlapped_dp_greedy_evaluation_keeps_weights_frozen(native_built):
    """the greedy evaluation under overlapped DP ran with the training lr on the delayed-
    update structs and moved the weights; now both ranks evaluate with frozen weights and continue training."""
    E, steps, world = 64, 5, 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _port(), E, steps, "bf16", d, True, True), nprocs=world,
                           join=True, start_method="spawn")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["params"], res[1]["params"]) and torch.isfinite(res[0]["params"]).all()
    assert res[0]["greedy"] == res[1]["greedy"]


def test_gloo_dp_split_graphs_match_eager(native_built):
    """gloo groups: capture_graph builds the two graphs around the host-side all-reduce (_capture_split);
    replaying them gives the eager trajectory bit for bit on both ranks."""
    E, steps, world = 64, 6, 2
    out = {}
    for graph in (False, True):
        with tempfile.TemporaryDirectory() as d:
            mp.start_processes(_worker, args=(world, _port(), E, steps, "bf16", d, False, False, graph),
                               nprocs=world, join=True, start_method="spawn")
            out[graph] = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert all(r["captured"] for r in out[True])
    for r in range(world):
        assert torch.equal(out[True][r]["params"], out[False][r]["params"])
        assert torch.equal(out[True][r]["budget"], out[False][r]["budget"])


def _rccl_capture_worker(_rank, port, out):
    """One rank over a real RCCL group: the sync-DP step (slab reduce -> all-reduce -> optimizer)
    captured in a multi-step HIP graph vs the same step launched eagerly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sharetrade.parallel.dist import DistContext, GradSync
    from sharetrade.trainer.engine import VectorEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {}
    for mode in ("eager", "graph"):
        cfg = _cfg("bf16")
        eng = VectorEngine(cfg, prices=_bank(256), device=dev, envs=256)
        # the DP code path (world_size > 1) over the 1-rank RCCL group
        eng.world_size = 2
        eng._sync = GradSync(DistContext(0, 2, 0, "nccl", dev, dist.group.WORLD), eng.layout.numel)
        if mode == "graph":
            assert eng.capture_graph(warmup=2, graph_steps=4)
            eng.run(9)                   # 2 x 4-step graph + 1 single-step graph
        else:
            eng.run(11)
        torch.cuda.synchronize()
        res[mode] = {"params": eng.params.cpu(), "budget": eng.state.budget.cpu(), "step": eng.step_count}
    torch.save(res, os.path.join(out, "cap.pt"))
    dist.destroy_process_group()


def test_sync_dp_step_captured_with_rccl_matches_eager(native_built):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rccl_capture_worker, args=(_port(), d), nprocs=1, join=True, start_method="spawn")
        res = torch.load(os.path.join(d, "cap.pt"), weights_only=True)
    assert res["eager"]["step"] == res["graph"]["step"] == 11
    assert torch.equal(res["eager"]["params"], res["graph"]["params"])
    assert torch.equal(res["eager"]["budget"], res["graph"]["budget"])
