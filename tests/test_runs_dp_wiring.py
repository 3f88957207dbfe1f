"""Data-parallel wiring of the config-4 / config-5 training runs (sharetrade/trainer/runs.py) on CPU,
gloo, world_size 2: a stand-in learner with the learners' DP surface (flat gradient, ``grad_sync``
hook, ``sync_params``, ``world_size``) shows that the run broadcasts rank 0's parameters, sums the
gradients of both ranks before every step, writes metrics on rank 0 only and checkpoints per rank.
The real learners' GPU counterpart is tests/test_gpu_learners_dp.py."""
import json
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Learner:
    """Plain SGD on a flat parameter vector; the gradient of iteration i on rank r is (r + 1) * (i + 1)."""

    def __init__(self, rank, world):
        self.world_size, self.rank = world, rank
        self.flat = torch.full((8,), float(10 * (rank + 1)))     # ranks start apart
        self.gflat = torch.zeros(8)
        self.grad_sync = None
        self.updates = 0

    def sync_params(self, ctx):
        from sharetrade.parallel.dist import broadcast_tensors

        broadcast_tensors(ctx, [self.flat])

    def capture(self):
        self._captured = True
        self.iteration(1)

    def iteration(self, n=1):
        self.gflat.fill_(float((self.rank + 1) * (self.updates + 1)))
        if self.grad_sync is not None:
            self.grad_sync(self.gflat)
        self.flat -= 0.5 * self.gflat
        self.updates += 1

    def state_dict(self):
        return {"flat": self.flat.clone(), "counters": torch.tensor([self.updates])}

    def stats_dict(self):
        return {"updates": self.updates}


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from sharetrade.config import preset_config
    from sharetrade.parallel.dist import DistContext
    from sharetrade.trainer.runs import run

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = DistContext(rank, world, 0, "gloo", torch.device("cpu"), dist.group.WORLD)
    d = _Learner(rank, world)
    res = run("recurrent", preset_config("recurrent"), 4, device=torch.device("cpu"), ctx=ctx, learner=d,
              metrics_path=os.path.join(out, f"m{rank}.jsonl"), log_every=2, ckpt_dir=os.path.join(out, "ck"),
              ckpt_every=4)
    torch.save({"flat": d.flat, "res_world": res["world_size"]}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_run_dp_broadcasts_sums_gradients_and_splits_outputs():
    from sharetrade.persist.checkpoint import CheckpointManager

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _port(), d), nprocs=world, join=True, start_method="spawn")
        r = [torch.load(os.path.join(d, f"r{k}.pt"), weights_only=True) for k in range(world)]
        # rank 0's start (10), then per iteration i the summed gradient (1 + 2) * (i + 1), lr 0.5
        want = 10.0 - 0.5 * sum(3.0 * (i + 1) for i in range(4))
        for k in range(world):
            assert r[k]["res_world"] == world
            assert torch.equal(r[k]["flat"], torch.full((8,), want))
        # metrics from rank 0 only; one checkpoint directory per rank
        assert os.path.exists(os.path.join(d, "m0.jsonl")) and not os.path.exists(os.path.join(d, "m1.jsonl"))
        recs = [json.loads(x) for x in open(os.path.join(d, "m0.jsonl"))]
        assert [x["iteration"] for x in recs] == [2, 4] and all(x["world_size"] == world for x in recs)
        for k in range(world):
            mgr = CheckpointManager(os.path.join(d, "ck", f"rank{k}"))
            assert [os.path.basename(p) for p in mgr.list()] == ["ckpt-000000000004.stck"]


def test_run_dp_rejects_a_learner_built_for_another_world():
    import pytest

    from sharetrade.config import preset_config
    from sharetrade.parallel.dist import DistContext
    from sharetrade.trainer.runs import run

    ctx = DistContext(0, 2, 0, "gloo", torch.device("cpu"), None)
    with pytest.raises(ValueError, match="world_size"):
        run("recurrent", preset_config("recurrent"), 1, device=torch.device("cpu"), ctx=ctx, learner=_Learner(0, 1))


def test_run_writes_a_chrome_trace(tmp_path):
    from sharetrade.config import preset_config
    from sharetrade.trainer.runs import run

    t = tmp_path / "trace.json"
    res = run("recurrent", preset_config("recurrent"), 3, device=torch.device("cpu"), learner=_Learner(0, 1),
              log_every=0, trace_path=str(t))
    assert res["iterations"] == 3
    assert "traceEvents" in json.loads(t.read_text())
