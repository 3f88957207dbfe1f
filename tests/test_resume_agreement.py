"""Data-parallel resume of the learner runs agrees on ONE step (CPU, gloo, 2 ranks).

A rank killed mid-save can leave another rank one checkpoint ahead; `runs.agreed_resume_step` takes
the MIN of every rank's newest valid checkpoint so all ranks restart at the same iteration (same
number of all-reduces, same parameters)."""
import datetime
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, root):
    import torch.distributed as dist

    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from sharetrade.parallel import dist as D
    from sharetrade.persist.checkpoint import CheckpointManager
    from sharetrade.trainer.runs import agreed_resume_step

    ctx = D.init(backend="gloo", device="cpu", timeout_s=30)
    mgr = CheckpointManager(os.path.join(root, f"rank{rank}"), interval=10)
    steps = (10, 20) if rank == 0 else (10, 20, 30)     # rank 1 saved once more before the kill
    for s in steps:
        mgr.save(s, {"w": torch.full((4,), float(s))}, {"kind": "deep"})
    got = agreed_resume_step(mgr, ctx)
    # a rank with no checkpoint at all: every rank starts fresh
    empty = CheckpointManager(os.path.join(root, f"empty{rank}"), interval=10)
    if rank == 1:
        empty.save(10, {"w": torch.zeros(1)}, {"kind": "deep"})
    got_empty = agreed_resume_step(empty, ctx)
    with open(os.path.join(root, f"out{rank}"), "w") as f:
        f.write(f"{got} {got_empty}")
    D.shutdown(ctx)


def test_ranks_agree_on_min_resume_step():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        outs = [open(os.path.join(d, f"out{r}")).read() for r in range(world)]
    assert outs == ["20 None", "20 None"], outs
