"""``--elastic N`` for the CLI training jobs (``engine``, ``deep``, ``recurrent``).

The reference wraps every rollout worker in a ``BackoffSupervisor`` and replaces dead ones
(`TrainerRouterActor.scala:46-58,101-102,116-120`).  For a multi-GPU CLI job the same duties fall to
:class:`~sharetrade.parallel.elastic.ElasticRunner`: the launching process (which never touches the GPU)
spawns one rank process per GPU; every rank publishes a heartbeat and its step (the progress mark) into
the launcher's store; a rank that exits non-zero, stops beating or stops making progress fails the
generation; the launcher kills the survivors (a communicator with a dead member cannot be repaired),
backs off, respawns the whole generation on a fresh port, and every rank resumes from the newest step
all ranks committed (sharded checkpoints; MIN over ranks) and continues to the same total step count.
RCCL / gloo collectives run with a finite timeout (``--pg-timeout``) and
``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``, so a peer blocked on a dead rank fails fast instead of hanging.
Fault injection: ``SHARETRADE_FAIL_AT`` / ``SHARETRADE_HANG_AT`` = ``rank:step[:generation]``.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional


def cli_worker(rank: int, world: int, generation: int, kind: str, cfg_dict: Dict[str, Any], kw: Dict[str, Any]) -> None:
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
    import torch

    from ..config import Config
    from . import dist as D
    from .elastic import Heartbeat, fail_point, heartbeat_store

    cfg = Config.from_dict(cfg_dict)
    device = kw.get("device", "cuda")
    if kw.get("same_device"):
        os.environ["LOCAL_RANK"] = "0"   # rehearsal: every rank on cuda:0
    if device == "cpu":
        torch.set_num_threads(1)
    ctx = D.init(backend=kw.get("backend"), device=device, timeout_s=float(kw.get("pg_timeout_s", 120.0)))
    hb = None
    store = heartbeat_store()
    if store is not None:
        hb = Heartbeat(store, rank, generation).start()

    def on_step(step: int) -> None:
        if hb is not None:
            hb.progress(step)
        fail_point(rank, step, generation)

    try:
        if kind == "engine":
            from ..trainer.loop import train

            res = train(cfg, int(kw["steps"]), device=ctx.device, envs=kw.get("envs"), metrics_path=kw.get("metrics"),
                        log_every=int(kw.get("log_every", 100)), ckpt_dir=kw["ckpt_dir"],
                        ckpt_every=int(kw["ckpt_every"]), resume=True, graph=bool(kw.get("graph", True)),
                        rank=ctx.rank, world_size=ctx.world_size, group=ctx.group, until=int(kw["steps"]),
                        on_step=on_step, final_dir=kw.get("final_dir"))
        else:
            from ..trainer.runs import run as run_learner

            lk = dict(kw.get("learner_kw") or {})
            res = run_learner(kind, cfg, int(kw["steps"]), device=ctx.device, metrics_path=kw.get("metrics"),
                              log_every=int(kw.get("log_every", 50)), ckpt_dir=kw["ckpt_dir"],
                              ckpt_every=int(kw["ckpt_every"]), resume=True, graph=bool(kw.get("graph", True)),
                              ctx=ctx, on_step=on_step, final_dir=kw.get("final_dir"), **lk)
        if ctx.is_main and kw.get("result_path"):
            import json

            with open(kw["result_path"], "w") as f:
                f.write(json.dumps(res, default=float))
    finally:
        if hb is not None:
            hb.stop()
        D.shutdown(ctx)


def run_elastic(kind: str, cfg, world: int, kw: Dict[str, Any], max_restarts: int = 3,
                stall_timeout_s: Optional[float] = 120.0, heartbeat_timeout_s: float = 30.0,
                gen_timeout_s: float = 24 * 3600.0):
    """Run ``kind`` on ``world`` rank processes under the elastic launcher; returns the ElasticResult."""
    from .elastic import ElasticRunner

    if not kw.get("ckpt_dir") or not int(kw.get("ckpt_every", 0)):
        raise ValueError("--elastic needs --ckpt-dir and --ckpt-every (a respawned generation resumes from them)")
    r = ElasticRunner(cli_worker, world, args=(kind, cfg.to_dict(), kw), max_restarts=max_restarts,
                      stall_timeout_s=stall_timeout_s, heartbeat_timeout_s=heartbeat_timeout_s,
                      gen_timeout_s=gen_timeout_s)
    return r.run()
