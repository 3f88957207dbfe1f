"""Data-parallel training worker with sharded checkpoints and resume.

One process per device (torchrun / :class:`~sharetrade.parallel.elastic.ElasticRunner`).
Each rank owns ``envs`` environments (its slice of the global env ids), all ranks
hold identical parameters (broadcast at start, flat-bucket gradient all-reduce
every step).  Every ``ckpt_every`` steps each rank writes its shard
``step-<S>/rank-<r>.stck`` (params + optimizer + its env state + counters) with the
deterministic C++ writer; rank 0 then publishes ``step-<S>/COMMIT``.  On start a
rank resumes from the newest committed step, so a respawned generation continues
bit-exactly where the failed one last checkpointed.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional

import torch

from ..config import Config
from ..persist import checkpoint as ck
from . import dist as D
from .elastic import Heartbeat, fail_point, heartbeat_store


def committed_steps(ckpt_dir: str):
    if not os.path.isdir(ckpt_dir):
        return []
    out = []
    for d in os.listdir(ckpt_dir):
        if d.startswith("step-") and os.path.exists(os.path.join(ckpt_dir, d, "COMMIT")):
            out.append(int(d[5:]))
    return sorted(out)


def save_shard(ckpt_dir: str, step: int, rank: int, eng) -> str:
    d = os.path.join(ckpt_dir, f"step-{step:09d}")
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, f"rank-{rank}.stck")
    ck.save(p, eng.state_dict(), {"step": step, "rank": rank, "world": eng.world_size})
    return p


def commit(ckpt_dir: str, step: int, world: int) -> None:
    d = os.path.join(ckpt_dir, f"step-{step:09d}")
    if all(os.path.exists(os.path.join(d, f"rank-{r}.stck")) for r in range(world)):
        with open(os.path.join(d, "COMMIT"), "w") as f:
            f.write(json.dumps({"step": step, "world": world}))


def dp_worker(rank: int, world: int, generation: int, cfg_dict: Dict[str, Any], steps: int, ckpt_dir: str,
              ckpt_every: int, envs: int, out_dir: str, device: str = "cpu", backend: Optional[str] = None,
              prices_seed: int = 11, T: int = 300) -> None:
    from ..data.prices import random_walk
    from ..trainer.engine import VectorEngine

    torch.set_num_threads(1)
    cfg = Config.from_dict(cfg_dict)
    ctx = D.init(backend=backend or ("gloo" if device == "cpu" else None), device=device)
    hb = None
    try:
        store = heartbeat_store()   # hosted by ElasticRunner's watchdog
        hb = Heartbeat(store, rank, generation).start() if store is not None else None
    except Exception:  # noqa: BLE001
        hb = None
    import numpy as np

    bank = torch.from_numpy(random_walk(T, 50.0, 0.02, prices_seed, n_series=envs * world).astype(np.float32))
    eng = VectorEngine(cfg, prices=bank[rank * envs:(rank + 1) * envs], device=ctx.device, rank=rank,
                       world_size=world, group=ctx.group, envs=envs,
                       backend="torch" if ctx.device.type == "cpu" else None)
    start = 0
    done = committed_steps(ckpt_dir)
    if done:
        start = done[-1]
        state, _ = ck.load(os.path.join(ckpt_dir, f"step-{start:09d}", f"rank-{rank}.stck"))
        eng.load_state_dict(state)
    eng.sync_params_from(0)        # re-dispatch: every rank continues from rank 0's learner state
    for step in range(start, steps):
        if hb is not None:
            hb.progress(step)
        fail_point(rank, step, generation)
        eng.step()
        s = step + 1
        if ckpt_every and s % ckpt_every == 0 and s < steps:
            eng.synchronize()
            save_shard(ckpt_dir, s, rank, eng)
            if ctx.is_distributed:
                torch.distributed.barrier()
            if rank == 0:
                commit(ckpt_dir, s, world)
            if ctx.is_distributed:
                torch.distributed.barrier()
    eng.synchronize()
    os.makedirs(out_dir, exist_ok=True)
    ck.save(os.path.join(out_dir, f"final-rank-{rank}.stck"), eng.state_dict(),
            {"generation": generation, "start": start})
    if hb is not None:
        hb.stop()
    D.shutdown(ctx)
