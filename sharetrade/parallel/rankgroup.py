"""The router fan-out as the multi-GPU data plane: one rank process per GPU, driven by the actors.

Reference (`TrainerRouterActor.scala:36,46-66,86-94,101-102,116-120,137-146`): the router broadcasts
``Train(data)`` to its rollout workers, death-watches them, replaces a dead worker and re-sends it
``Train``, and answers ``GetAvg`` / ``GetStd`` by scatter-gathering the workers' final portfolios.
Here every routee is backed by one RANK PROCESS of a ``torch.distributed`` group (RCCL over xGMI on
MI355X, gloo on the CPU); the ranks run their env slices of one synchronous data-parallel learner:

=============================================  ===================================================
reference                                      here
=============================================  ===================================================
``router.route(Train(d))`` (broadcast)         ``("train", prices, ...)`` to every rank; each rank
                                               builds its engine over the series and starts from
                                               rank 0's weights (``broadcast``)
worker's episode + ``UpdateQ`` to ONE learner  ``T - H`` engine steps per rank, gradients summed by
                                               ``all_reduce`` every step (captured in the step's HIP
                                               graph on RCCL)
``Trained`` from every worker                  ``all_done`` (MIN all-reduce) at the episode's end
``GetAvg`` / ``GetStd`` scatter-gather         ``global_mean_std`` (one all-reduce of n, Sx, Sxx)
``Terminated`` -> new child + ``Train``        a dead rank (exit status, or no progress within the
                                               stall timeout) fails the generation: every rank is
                                               killed (a communicator with a dead member cannot be
                                               repaired), a fresh generation is spawned on a new port
                                               after a backoff and resumes from the newest step every
                                               rank has COMMITTED (sharded checkpoints, MIN over ranks)
=============================================  ===================================================

:class:`RankGroup` owns the processes (spawned as fresh interpreters: the parent never touches the
GPU); ``sharetrade/trainer/dp_actors.py`` puts the actor API on top of it.
"""
from __future__ import annotations

import os
import time
import zlib
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ..actors.backoff import calculate_delay
from .elastic import fail_point, free_port


# ---------------------------------------------------------------------------------- rank process
def _rank_entry(rank: int, world: int, gen: int, port: int, conn, cfg_dict: Dict[str, Any], device: str,
                backend: Optional[str], same_device: bool, pg_timeout_s: float) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(0 if same_device else rank), SHARETRADE_GENERATION=str(gen))
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
    import torch

    from ..config import Config
    from . import dist as D

    if device == "cpu":
        torch.set_num_threads(1)
    ctx = D.init(backend=backend, device=device, timeout_s=pg_timeout_s)
    cfg = Config.from_dict(cfg_dict)
    params = None
    try:
        while True:
            msg = conn.recv()
            if msg[0] == "stop":
                break
            if msg[0] == "train":
                _, prices, envs, ckpt_dir, ckpt_every, progress_every, out_dir = msg
                res, params = _train_episode(rank, world, gen, ctx, cfg, prices, envs, ckpt_dir, ckpt_every,
                                             progress_every, out_dir, conn, params)
                conn.send(("trained", rank, res))
    finally:
        D.shutdown(ctx)


def _train_episode(rank, world, gen, ctx, cfg, prices: np.ndarray, envs: int, ckpt_dir: str, ckpt_every: int,
                   progress_every: int, out_dir: Optional[str], conn, params):
    import torch

    from ..persist import checkpoint as ck
    from ..trainer.engine import VectorEngine
    from ..trainer.loop import _load_committed_shard, _save_sharded
    from . import dist as D

    bank = torch.from_numpy(np.asarray(prices, dtype=np.float32))[None, :].expand(envs, -1).contiguous()
    eng = VectorEngine(cfg, prices=bank, device=ctx.device, rank=rank, world_size=world, group=ctx.group, envs=envs,
                       backend="torch" if ctx.device.type == "cpu" else None, params=params)
    steps = eng.T - eng.H
    start = 0
    st = _load_committed_shard(ckpt_dir, rank, eng.device, ctx.group) if world > 1 else None
    if st is not None:
        eng.load_state_dict(st)
        start = eng.step_count
    eng.sync_params_from(0)          # re-dispatch: every rank continues from rank 0's learner state
    if eng.backend == "native" and cfg.engine.graph:
        # the synchronous DP step (kernel, slab reduce, RCCL all-reduce, optimizer) in HIP graphs; every
        # rank captures (no collective runs during a capture) and the ranks vote: a capture failure on
        # one rank sends every rank down the eager path (gloo groups stay eager)
        from ..trainer.benchkit import capture_with_vote

        capture_with_vote(eng, rank, world, ctx.group, warmup=0)
    step = start
    while step < steps:
        # one multi-step graph replay at a time (VectorEngine.run), never across a progress / checkpoint
        # point; the fault-injection points of every step of it are checked before it runs
        nxt = min(steps, step + max(1, int(cfg.engine.graph_steps)))
        for every in (progress_every, ckpt_every):
            if every:
                nxt = min(nxt, (step // every + 1) * every)
        for s_ in range(step, nxt):
            fail_point(rank, s_, gen)
        eng.run(nxt - step)
        step = s = nxt
        if progress_every and s % progress_every == 0:
            conn.send(("progress", rank, s))
        if ckpt_every and s % ckpt_every == 0 and s < steps:
            _save_sharded(ckpt_dir, s, rank, world, eng, ctx.group)
    eng.synchronize()
    final = eng.final_portfolios()
    stats = D.global_mean_std(ctx, final)
    done = D.all_done(ctx, bool((~torch.isnan(final)).all()))
    p = eng.params.detach().cpu()
    res = {"mean": stats["mean"], "std": stats["std"], "n": stats["n"], "all_done": done, "steps": steps,
           "start": start, "generation": gen, "rank_mean": float(final.double().mean()),
           "params_crc": zlib.crc32(p.numpy().tobytes()), "step_count": eng.step_count}
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        ck.save(os.path.join(out_dir, f"final-rank-{rank}.stck"), eng.state_dict(), {"generation": gen, "start": start})
    return res, p


# ---------------------------------------------------------------------------------- the group
@dataclass
class RankDeath:
    generation: int
    rank: int
    reason: str


@dataclass
class EpisodeResult:
    ranks: List[Dict[str, Any]]
    generations: int
    deaths: List[RankDeath] = field(default_factory=list)

    @property
    def global_stats(self) -> Dict[str, float]:
        r0 = self.ranks[0]
        return {"mean": r0["mean"], "std": r0["std"], "n": r0["n"]}


class RankGroup:
    """``world`` rank processes of one DP group (generation ``gen``), respawned as a whole on failure."""

    def __init__(self, world: int, cfg_dict: Dict[str, Any], device: str = "cpu", backend: Optional[str] = None,
                 same_device: bool = False, max_restarts: int = 3, min_backoff_s: float = 0.05,
                 max_backoff_s: float = 2.0, jitter: float = 0.2, stall_timeout_s: float = 120.0,
                 pg_timeout_s: float = 120.0, on_death: Optional[Callable[[RankDeath], None]] = None):
        self.world, self.cfg_dict, self.device, self.backend = world, cfg_dict, device, backend
        self.same_device = same_device
        self.max_restarts = max_restarts
        self.min_b, self.max_b, self.jitter = min_backoff_s, max_backoff_s, jitter
        self.stall = stall_timeout_s
        self.pg_timeout = pg_timeout_s
        self.on_death = on_death
        self.gen = -1
        self.procs: List[Any] = []
        self.conns: List[Any] = []
        self.deaths: List[RankDeath] = []

    # ------------------------------------------------------------------ processes
    def _spawn(self) -> None:
        import torch.multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.gen += 1
        port = free_port()
        self.procs, self.conns = [], []
        for r in range(self.world):
            parent_end, child_end = ctx.Pipe(duplex=True)
            p = ctx.Process(target=_rank_entry, args=(r, self.world, self.gen, port, child_end, self.cfg_dict,
                                                      self.device, self.backend, self.same_device, self.pg_timeout),
                            daemon=True)
            p.start()
            child_end.close()
            self.procs.append(p)
            self.conns.append(parent_end)

    def _kill(self) -> None:
        for p in self.procs:
            if p.exitcode is None:
                p.kill()
        for p in self.procs:
            p.join(timeout=30)
        for c in self.conns:
            try:
                c.close()
            except OSError:
                pass
        self.procs, self.conns = [], []

    def alive(self) -> bool:
        return bool(self.procs) and all(p.exitcode is None for p in self.procs)

    # ------------------------------------------------------------------ one episode
    def run_episode(self, prices: np.ndarray, envs: int, ckpt_dir: str, ckpt_every: int = 0,
                    progress_every: int = 10, out_dir: Optional[str] = None) -> EpisodeResult:
        """Every rank plays one episode over ``prices`` with ``envs`` envs; on a rank's death the whole
        generation is replaced and resumes from the newest step every rank committed."""
        deaths: List[RankDeath] = []
        first_gen = self.gen + 1 if not self.alive() else self.gen
        for attempt in range(self.max_restarts + 1):
            if attempt:
                time.sleep(calculate_delay(attempt - 1, self.min_b, self.max_b, self.jitter))
            if not self.alive():
                self._kill()
                self._spawn()
            for c in self.conns:
                c.send(("train", np.asarray(prices, dtype=np.float32), int(envs), ckpt_dir, int(ckpt_every),
                        int(progress_every), out_dir))
            results: Dict[int, Dict[str, Any]] = {}
            last = time.monotonic()
            death: Optional[RankDeath] = None
            while len(results) < self.world and death is None:
                for r, (p, c) in enumerate(zip(self.procs, self.conns)):
                    try:
                        while c.poll():
                            m = c.recv()
                            last = time.monotonic()
                            if m[0] == "trained":
                                results[m[1]] = m[2]
                    except (EOFError, OSError):
                        pass
                    if r not in results and p.exitcode is not None:
                        death = RankDeath(self.gen, r, f"exit status {p.exitcode}")
                        break
                if death is None and time.monotonic() - last > self.stall:
                    death = RankDeath(self.gen, -1, f"no progress for {self.stall:.0f} s")
                if death is None:
                    time.sleep(0.005)
            if death is None:
                return EpisodeResult([results[r] for r in range(self.world)], self.gen - first_gen + 1, deaths)
            deaths.append(death)
            self.deaths.append(death)
            if self.on_death is not None:
                self.on_death(death)
            self._kill()      # peers are blocked in a collective with the dead rank: tear the generation down
        raise RuntimeError(f"rank group gave up after {self.max_restarts} restarts: {deaths}")

    def close(self) -> None:
        for c in self.conns:
            try:
                c.send(("stop",))
            except (OSError, BrokenPipeError):
                pass
        deadline = time.monotonic() + 30
        for p in self.procs:
            p.join(timeout=max(0.1, deadline - time.monotonic()))
        self._kill()
