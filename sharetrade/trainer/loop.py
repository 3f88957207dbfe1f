"""Training loop around :class:`VectorEngine`: metrics, periodic checkpoints, resume, traces.

Used by ``python -m sharetrade engine`` (single process or one rank of a
torchrun / ElasticRunner job)."""
from __future__ import annotations

import os
import time
from typing import Any, Callable, Dict, Optional

import torch

from ..config import Config
from ..persist.checkpoint import CheckpointManager, load as load_ckpt
from ..utils.metrics import MetricsLogger, WindowStats
from .engine import VectorEngine


def train(cfg: Config, steps: int, device: Optional[torch.device] = None, envs: Optional[int] = None,
          metrics_path: Optional[str] = None, log_every: int = 100, ckpt_dir: Optional[str] = None,
          ckpt_every: int = 0, resume: bool = False, trace_path: Optional[str] = None, graph: bool = True,
          rank: int = 0, world_size: int = 1, group=None, until: Optional[int] = None,
          on_step: Optional[Callable[[int], None]] = None, final_dir: Optional[str] = None) -> Dict[str, Any]:
    """``steps`` more steps (or, with ``until``, up to that total step count -- a resumed elastic
    generation finishes the same job).  The steps between two logging / checkpoint points run as whole
    multi-step graph replays (``VectorEngine.run``).  ``on_step(step)`` (fault injection and the
    heartbeat's progress mark of ``--elastic`` jobs) is called for every step of the next replay before
    that replay runs; with it, one replay (``engine.graph_steps`` steps) runs at a time.  ``final_dir``: each
    rank writes its final state there (``final-rank-<r>.stck``).

    Several ranks (one process per GPU, RCCL): the synchronous DP step -- kernel, slab reduce, all-reduce,
    optimizer -- is captured in HIP graphs on every rank; the ranks vote (MIN all-reduce) so that a
    capture failure on one rank sends every rank down the eager path with the same collectives."""
    eng = VectorEngine(cfg, device=device, envs=envs, rank=rank, world_size=world_size, group=group)
    # one process: CheckpointManager files; several ranks: one shard per rank per step, committed by
    # rank 0 after a barrier (parallel/dp_train.py) -- every rank owns different envs / price banks
    sharded = world_size > 1
    mgr = CheckpointManager(ckpt_dir, interval=ckpt_every) if ckpt_dir and not sharded else None
    if ckpt_dir and resume:
        if sharded:
            st = _load_committed_shard(ckpt_dir, rank, eng.device, group)
            if st is not None:
                eng.load_state_dict(st)
        elif mgr.latest():
            st, _ = load_ckpt(mgr.latest())
            eng.load_state_dict(st)
    eng.sync_params_from(0)
    if graph and eng.backend == "native":
        from .benchkit import capture_with_vote

        capture_with_vote(eng, rank, world_size, group, warmup=0 if world_size > 1 else 1)
    if eng._sync is not None:
        eng._sync.enable_timing()          # metrics: mean all-reduce ms per logging window
    ml = MetricsLogger(metrics_path)
    ws = WindowStats()
    ws.window(eng.stats_dict(), eng.step_count, eng.E, world_size)
    prof = None
    if trace_path:
        acts = [torch.profiler.ProfilerActivity.CPU]
        if eng.device.type == "cuda":
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        prof = torch.profiler.profile(activities=acts)
        prof.__enter__()
    t0 = time.perf_counter()
    start = eng.step_count
    target = int(until) if until is not None else start + steps
    while eng.step_count < target:
        # whole graph replays up to the next logging / checkpoint point; with ``on_step`` (the heartbeat's
        # progress mark and the fault-injection points of --elastic jobs) at most one multi-step replay
        # at a time, on_step called for every step of it before it runs
        nxt = target
        for every in (log_every, ckpt_every):
            if every:
                nxt = min(nxt, (eng.step_count // every + 1) * every)
        if on_step is not None:
            nxt = min(nxt, eng.step_count + max(1, int(eng.cfg.engine.graph_steps)))
            for s_ in range(eng.step_count, nxt):
                on_step(s_)
        eng.run(nxt - eng.step_count)
        s = eng.step_count
        if log_every and s % log_every == 0:
            eng.synchronize()
            rec = ws.window(eng.stats_dict(), s, eng.E, world_size)
            if eng._sync is not None:
                ms = eng._sync.pop_timing_ms()
                if ms is not None:
                    rec["allreduce_ms"] = ms
            ml.log(rec)
        if mgr and mgr.should_save(s):
            eng.synchronize()
            mgr.save(s, eng.state_dict(), {"kind": "VectorEngine"})
        elif sharded and ckpt_dir and ckpt_every and s % ckpt_every == 0:
            _save_sharded(ckpt_dir, s, rank, world_size, eng, group)
    eng.synchronize()
    dt = time.perf_counter() - t0
    if final_dir:
        from ..persist import checkpoint as ck

        os.makedirs(final_dir, exist_ok=True)
        ck.save(os.path.join(final_dir, f"final-rank-{rank}.stck"), eng.state_dict(), {"rank": rank})
    steps = eng.step_count - start
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(os.path.dirname(os.path.abspath(trace_path)) or ".", exist_ok=True)
        prof.export_chrome_trace(trace_path)
    ml.close()
    return {"backend": eng.backend, "kernel": eng.kernel, "envs": eng.E, "steps": steps,
            "env_steps_per_s": eng.E * world_size * steps / dt, "seconds": dt, **eng.stats_dict(),
            **eng.portfolio_summary()}


def _save_sharded(ckpt_dir: str, step: int, rank: int, world: int, eng: VectorEngine, group, keep: int = 3) -> None:
    """Every rank writes its shard (``state_dict`` -- and so ``flush_pending`` -- runs on every rank,
    keeping the overlapped-DP schedule identical across ranks); rank 0 commits after a barrier."""
    import shutil

    import torch.distributed as dist

    from ..parallel.dp_train import commit, committed_steps, save_shard

    eng.synchronize()
    save_shard(ckpt_dir, step, rank, eng)
    dist.barrier(group=group)
    if rank == 0:
        commit(ckpt_dir, step, world)
        for old in committed_steps(ckpt_dir)[:-keep]:
            shutil.rmtree(os.path.join(ckpt_dir, f"step-{old:09d}"), ignore_errors=True)
    dist.barrier(group=group)


def _load_committed_shard(ckpt_dir: str, rank: int, device: torch.device, group):
    """This rank's shard of the newest step every rank sees committed (MIN over ranks)."""
    import torch.distributed as dist

    from ..parallel.dp_train import committed_steps

    done = committed_steps(ckpt_dir)
    t = torch.tensor([done[-1] if done else -1], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    step = int(t[0])
    if step < 0:
        return None
    st, meta = load_ckpt(os.path.join(ckpt_dir, f"step-{step:09d}", f"rank-{rank}.stck"))
    if int(meta.get("rank", rank)) != rank:
        raise RuntimeError(f"shard for rank {rank} holds rank {meta.get('rank')}")
    return st
