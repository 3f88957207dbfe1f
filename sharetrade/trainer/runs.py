"""Training runs of the north-star learners (BASELINE configs 4 and 5) with the same run-level services
as the vectorised engine (`trainer/loop.py`): JSONL metrics, periodic checkpoints with retention,
bit-reproducible resume.

* ``deep``      -- :class:`~sharetrade.trainer.deep.DeepDQN` (4x1024 MLP, 1M-transition HBM replay);
* ``recurrent`` -- :class:`~sharetrade.trainer.recurrent.RecurrentDQN` (GRU(256), MX-fp8 actor).

One *iteration* is what the benchmarks time: one act step (deep) or one actor launch of S bars
(recurrent) plus one learner update, captured into HIP graphs after the first (eager) iteration.
A checkpoint written after iteration k holds the learner's whole state (`state_dict`); resuming
loads it and continues with iteration k+1.  The reference's `saveSnapshot` stub
(`QDecisionPolicyActor.scala:91-93`) is the model for the interval semantics (every N, not at 0).

Data parallel (``ctx`` from :func:`sharetrade.parallel.dist.init`, one process per GPU under
``torch.distributed.run``): every rank runs its own envs and replay (seed + rank), starts from rank 0's
parameters, and sums its gradients with the others' (one flat bucket, RCCL all-reduce) before each Adam
step, so the parameters stay identical on all ranks -- the reference's many workers feeding ONE shared
policy (`TrainerRouterActor.scala`), with synchronous gradient averaging in place of the shared actor.
Metrics come from rank 0 (its own envs); each rank checkpoints its own state under ``rank<r>/``.
"""
from __future__ import annotations

import os
import time
from typing import Any, Dict, Optional

import torch

from ..config import Config
from ..persist.checkpoint import CheckpointManager, load as load_ckpt
from ..utils.metrics import MetricsLogger


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def agreed_resume_step(mgr: CheckpointManager, ctx=None) -> Optional[int]:
    """The step every rank resumes from: this rank's newest valid checkpoint, MIN over ranks.

    A rank killed mid-save (the ElasticRunner tears a failed generation down with SIGKILL) can leave
    some ranks one checkpoint ahead of others; each loading its own newest file would restart the
    ranks at different iteration counts -- different numbers of all-reduces (a hang) and different
    parameters.  Retention keeps ``mgr.keep`` files per rank, so the MIN step is still on disk
    everywhere.  None: some rank has no checkpoint (every rank starts fresh)."""
    latest = mgr.latest()
    mine = int(os.path.basename(latest)[5:-5]) if latest else -1
    if ctx is not None and ctx.is_distributed:
        import torch.distributed as dist

        t = torch.tensor([mine], dtype=torch.int64, device=ctx.device if ctx.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.group)
        mine = int(t.item())
    return None if mine < 0 else mine


def build(kind: str, cfg: Config, device: torch.device, **kw):
    if kind == "deep":
        from .deep import DeepDQN

        kw.setdefault("overlap_act", True)
        return DeepDQN(cfg, device, **kw)
    if kind == "recurrent":
        from .recurrent import RecurrentDQN

        kw.setdefault("overlap_act", True)
        return RecurrentDQN(cfg, device, **kw)
    raise ValueError(f"unknown learner {kind!r}")


def run(kind: str, cfg: Config, iterations: int, device: Optional[torch.device] = None,
        metrics_path: Optional[str] = None, log_every: int = 50, ckpt_dir: Optional[str] = None,
        ckpt_every: int = 0, resume: bool = False, graph: bool = True, learner=None, ctx=None,
        bucket_mb: float = 64.0, capture_sync: bool = True, layer_overlap: bool = True,
        trace_path: Optional[str] = None, on_step=None, final_dir: Optional[str] = None,
        **learner_kw) -> Dict[str, Any]:
    """Run ``iterations`` act + update iterations (counting any restored ones); returns final stats.
    ``on_step(i)`` runs before every iteration (``--elastic``: fault injection + heartbeat progress);
    ``final_dir``: each rank writes its final learner state there (``final-rank-<r>.stck``)."""
    dp = ctx is not None and ctx.is_distributed
    dev = device or (ctx.device if ctx is not None else torch.device("cuda", 0))
    if dp:
        if learner is None:           # own envs / replay per rank; parameters come from rank 0
            seed = learner_kw.pop("seed", None)
            learner_kw["seed"] = (cfg.agent.seed if seed is None else int(seed)) + ctx.rank
            learner_kw["world_size"] = ctx.world_size
            if kind == "deep":
                learner_kw.setdefault("bank_seed", ctx.rank)     # each rank its own price series
        if ckpt_dir:
            ckpt_dir = os.path.join(ckpt_dir, f"rank{ctx.rank}")
    d = learner if learner is not None else build(kind, cfg, dev, **learner_kw)
    if dp:
        if d.world_size != ctx.world_size:
            raise ValueError(f"learner built for world_size={d.world_size}, the group has {ctx.world_size}")
        from ..parallel.dist import GradSync

        gflat = d.grad_flat if kind == "deep" else d.gflat
        d.grad_sync = GradSync(ctx, gflat.numel(), bucket_mb=bucket_mb).all_reduce
        if ctx.backend == "nccl" and capture_sync:
            # RCCL collectives capture into HIP graphs: keep the all-reduce inside the update graph
            # (config 4: per layer on a comm stream, overlapped with the rest of the backward)
            import torch.distributed as dist

            d.capture_sync = True
            if kind == "deep" and layer_overlap:
                d.layer_sync = lambda t: dist.all_reduce(t, group=ctx.group)
        d.sync_params(ctx)
    if dp and not ctx.is_main:
        metrics_path = None
    mgr = CheckpointManager(ckpt_dir, interval=ckpt_every) if ckpt_dir else None
    done = 0
    if mgr is not None and resume:
        step = agreed_resume_step(mgr, ctx if dp else None)
        if step is not None:
            path = mgr.path_for(step)
            if not os.path.exists(path):
                raise RuntimeError(f"rank {ctx.rank if dp else 0}: the agreed resume step {step} is not in {mgr.dir} "
                                   f"(retention kept {mgr.list()})")
            st, meta = load_ckpt(path)
            if meta.get("kind") != kind:
                raise ValueError(f"checkpoint is a {meta.get('kind')!r} run, not {kind!r}")
            d.load_state_dict(st)
            done = int(meta["step"])
    ml = MetricsLogger(metrics_path)
    prof = None
    if trace_path and (not dp or ctx.is_main):      # Chrome trace of the run (host spans + GPU kernels)
        acts = [torch.profiler.ProfilerActivity.CPU]
        if dev.type == "cuda":
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        prof = torch.profiler.profile(activities=acts)
        prof.__enter__()
    t0 = time.perf_counter()
    last_t, last_i = t0, done

    def one() -> None:
        nonlocal done
        if graph and not getattr(d, "_captured", False):
            d.capture()                  # one eager warm-up iteration (counted), then the graphs
        else:
            d.iteration(1)
        done += 1

    while done < iterations:
        if on_step is not None:
            on_step(done)
        one()
        if mgr is not None and mgr.should_save(done):
            _sync(dev)
            mgr.save(done, d.state_dict(), {"kind": kind, "config": cfg.to_dict()})
        if log_every and done % log_every == 0:
            _sync(dev)
            now = time.perf_counter()
            s = d.stats_dict()
            rec = dict(kind=kind, iteration=done, it_per_s=(done - last_i) / max(now - last_t, 1e-9),
                       world_size=ctx.world_size if dp else 1, **s)
            ml.log(rec)
            last_t, last_i = now, done
    _sync(dev)
    if final_dir:
        from ..persist import checkpoint as ck

        os.makedirs(final_dir, exist_ok=True)
        ck.save(os.path.join(final_dir, f"final-rank-{ctx.rank if dp else 0}.stck"), d.state_dict(), {"kind": kind})
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(os.path.dirname(os.path.abspath(trace_path)) or ".", exist_ok=True)
        prof.export_chrome_trace(trace_path)
    out = dict(kind=kind, iterations=done, wall_s=time.perf_counter() - t0, world_size=ctx.world_size if dp else 1,
               **d.stats_dict())
    ml.close()
    return out
