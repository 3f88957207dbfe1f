"""Failure detection, elastic recovery and fault injection for multi-process runs.

Reference: rollout workers are wrapped in a ``BackoffSupervisor``
and death-watched by the router; a ``Terminated`` child is replaced
(`TrainerRouterActor.scala:46-64,101-102,116-120,141-146`) and, in the trained
state, ``StartTraining`` is re-broadcast.  Across processes the same duties are:

* **detect** — every rank publishes a liveness heartbeat (a thread) and a
  progress mark (its training step, from the main loop) into a store hosted by the
  launcher; the launcher's :class:`Watchdog` flags a rank whose heartbeat goes stale
  (process gone or frozen) or whose progress stops advancing (main loop hung, e.g.
  in a collective with a dead or stuck peer -- RCCL just blocks, so a timeout is the
  only signal).  The launcher also sees a worker's exit status / signal;
* **replace** — :class:`ElasticRunner` tears the whole generation down (a
  communicator with a dead member cannot be repaired), re-rendezvouses on a
  fresh port with generation ``g+1`` and respawns every rank (backoff between
  attempts, like the reference's 3 s .. 1 min backoff supervisor);
* **re-dispatch** — workers resume from the newest checkpoint written by rank 0
  (deterministic C++ writer) and rank 0's weights/optimizer state are broadcast,
  the analogue of re-sending ``Train`` to the replacement routee;
* **inject** — ``SHARETRADE_FAIL_AT="rank:step[:generation]"`` makes a worker
  die at a given step (``os._exit``), ``SHARETRADE_HANG_AT`` (same syntax) makes it
  hang there (alive, heartbeat thread still beating, no progress), :func:`kill_worker`
  SIGKILLs a pid.
"""
from __future__ import annotations

import os
import signal
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch.multiprocessing as mp

from ..actors.backoff import calculate_delay


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---------------------------------------------------------------------- fault injection
def _spec_hits(var: str, rank: int, step: int, generation: int) -> bool:
    spec = os.environ.get(var, "")
    if not spec:
        return False
    parts = [int(x) for x in spec.split(":")]
    g = parts[2] if len(parts) > 2 else 0
    return parts[0] == rank and parts[1] == step and g == generation


def fail_point(rank: int, step: int, generation: int = 0) -> None:
    """Die abruptly if ``SHARETRADE_FAIL_AT`` names this rank/step (and generation); hang
    (sleep forever, heartbeat thread alive) if ``SHARETRADE_HANG_AT`` does."""
    if _spec_hits("SHARETRADE_FAIL_AT", rank, step, generation):
        os._exit(17)
    if _spec_hits("SHARETRADE_HANG_AT", rank, step, generation):
        while True:
            time.sleep(3600)


def kill_worker(pid: int, sig: int = signal.SIGKILL) -> None:
    os.kill(pid, sig)


# ---------------------------------------------------------------------- heartbeat / watchdog
class Heartbeat:
    """Publishes ``hb/<gen>/<rank> = time`` into a ``torch.distributed.Store`` periodically."""

    def __init__(self, store, rank: int, generation: int = 0, interval_s: float = 0.5):
        self.store, self.rank, self.gen, self.interval = store, rank, generation, interval_s
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="heartbeat", daemon=True)

    def key(self, rank: int) -> str:
        return f"hb/{self.gen}/{rank}"

    def beat(self) -> None:
        self.store.set(self.key(self.rank), repr(time.time()))

    def progress(self, step: int) -> None:
        """Main-loop progress mark (the liveness thread keeps beating even when the loop hangs)."""
        self.store.set(f"prog/{self.gen}/{self.rank}", f"{int(step)} {time.time()!r}")

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            try:
                self.beat()
            except Exception:  # noqa: BLE001 - store gone: the run is being torn down
                return

    def start(self) -> "Heartbeat":
        self.beat()
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()


class Watchdog:
    """Flags peers whose heartbeat is older than ``timeout_s`` or -- when ``stall_timeout_s`` is
    set -- whose progress mark has not advanced for that long (calls ``on_dead(rank)``)."""

    def __init__(self, store, world_size: int, generation: int = 0, timeout_s: float = 5.0,
                 on_dead: Optional[Callable[[int], None]] = None, poll_s: float = 0.5,
                 stall_timeout_s: Optional[float] = None):
        self.store, self.world, self.gen = store, world_size, generation
        self.timeout, self.poll, self.stall = timeout_s, poll_s, stall_timeout_s
        self.on_dead = on_dead
        self.dead: List[int] = []
        # ranks whose process has exited cleanly: their heartbeat goes stale by design, never flag them
        # (a peer still committing its last checkpoint would otherwise fail a finished generation)
        self.finished: set = set()
        self._last: Dict[int, tuple] = {}       # rank -> (progress value, local time it last changed)
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="watchdog", daemon=True)

    def _get(self, key: str) -> Optional[str]:
        try:
            if not self.store.check([key]):
                return None
            return self.store.get(key).decode()
        except Exception:  # noqa: BLE001
            return None

    def check(self) -> List[int]:
        now = time.time()
        dead = []
        for r in range(self.world):
            if r in self.finished:
                continue
            v = self._get(f"hb/{self.gen}/{r}")
            if v is not None and now - float(v) > self.timeout:
                dead.append(r)
                continue
            if self.stall is None:
                continue
            p = self._get(f"prog/{self.gen}/{r}")
            if p is None:
                continue
            step = p.split()[0]
            seen = self._last.get(r)
            if seen is None or seen[0] != step:
                self._last[r] = (step, now)
            elif now - seen[1] > self.stall:
                dead.append(r)
        return dead

    def _run(self) -> None:
        while not self._stop.wait(self.poll):
            for r in self.check():
                if r not in self.dead:
                    self.dead.append(r)
                    if self.on_dead:
                        self.on_dead(r)

    def start(self) -> "Watchdog":
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()


# ---------------------------------------------------------------------- elastic launcher
@dataclass
class GenerationResult:
    generation: int
    exitcodes: Dict[int, Optional[int]]
    ok: bool
    seconds: float


@dataclass
class ElasticResult:
    ok: bool
    generations: List[GenerationResult] = field(default_factory=list)
    flagged: List[tuple] = field(default_factory=list)   # (generation, rank) flagged dead / hung by the watchdog

    @property
    def restarts(self) -> int:
        return max(0, len(self.generations) - 1)


def heartbeat_store():
    """Client of the launcher-hosted heartbeat store (``SHARETRADE_HB_ADDR``), or None."""
    addr = os.environ.get("SHARETRADE_HB_ADDR", "")
    if not addr:
        return None
    import datetime

    import torch.distributed as dist

    host, port = addr.rsplit(":", 1)
    return dist.TCPStore(host, int(port), is_master=False, timeout=datetime.timedelta(seconds=30))


def _entry(rank: int, fn, world: int, port: int, gen: int, args: tuple, env: Dict[str, str]) -> None:
    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHARETRADE_GENERATION=str(gen))
    fn(rank, world, gen, *args)


class ElasticRunner:
    """Run ``fn(rank, world, generation, *args)`` on ``world`` processes; on any
    failure kill the generation and respawn it (up to ``max_restarts``)."""

    def __init__(self, fn, world: int, args: tuple = (), max_restarts: int = 3, min_backoff_s: float = 0.05,
                 max_backoff_s: float = 2.0, jitter: float = 0.2, gen_timeout_s: float = 600.0,
                 env: Optional[Dict[str, str]] = None, stall_timeout_s: Optional[float] = 60.0,
                 heartbeat_timeout_s: float = 10.0):
        self.fn, self.world, self.args = fn, world, args
        self.max_restarts = max_restarts
        self.min_b, self.max_b, self.jitter = min_backoff_s, max_backoff_s, jitter
        self.gen_timeout = gen_timeout_s
        self.stall_timeout = stall_timeout_s          # None: no watchdog (exit codes + gen_timeout only)
        self.hb_timeout = heartbeat_timeout_s
        self.env = dict(env or {})
        self.flagged: List[tuple] = []              # (generation, rank) the watchdog declared dead / hung

    def run(self) -> ElasticResult:
        res = ElasticResult(ok=False, flagged=self.flagged)
        ctx = mp.get_context("spawn")
        for gen in range(self.max_restarts + 1):
            if gen:
                time.sleep(calculate_delay(gen - 1, self.min_b, self.max_b, self.jitter))
            port = free_port()
            env = dict(self.env)
            store = wd = None
            if self.stall_timeout is not None:
                # the launcher hosts the heartbeat store: it outlives any worker (rank 0 included)
                import torch.distributed as dist

                hb_port = free_port()
                store = dist.TCPStore("127.0.0.1", hb_port, is_master=True, wait_for_workers=False)
                env["SHARETRADE_HB_ADDR"] = f"127.0.0.1:{hb_port}"
                wd = Watchdog(store, self.world, gen, timeout_s=self.hb_timeout, poll_s=0.25,
                              stall_timeout_s=self.stall_timeout).start()
            t0 = time.perf_counter()
            procs = [ctx.Process(target=_entry, args=(r, self.fn, self.world, port, gen, self.args, env),
                                 daemon=False) for r in range(self.world)]
            for p in procs:
                p.start()
            failed = False
            deadline = time.monotonic() + self.gen_timeout
            while True:
                codes = [p.exitcode for p in procs]
                if any(c not in (None, 0) for c in codes):
                    failed = True
                    break
                if all(c == 0 for c in codes):
                    break
                if wd is not None:
                    wd.finished.update(r for r, c in enumerate(codes) if c == 0)
                    live_dead = [r for r in wd.dead if codes[r] != 0]
                    if live_dead:
                        self.flagged.extend((gen, r) for r in live_dead)
                        failed = True
                        break
                if time.monotonic() > deadline:
                    failed = True
                    break
                time.sleep(0.02)
            if wd is not None:
                wd.stop()
            if failed:
                # peers are likely blocked in a collective with the dead rank: tear down
                for p in procs:
                    if p.exitcode is None:
                        p.kill()
            for p in procs:
                p.join(timeout=30)
            del store
            gr = GenerationResult(gen, {r: p.exitcode for r, p in enumerate(procs)}, not failed,
                                  time.perf_counter() - t0)
            res.generations.append(gr)
            if not failed:
                res.ok = True
                return res
        return res
