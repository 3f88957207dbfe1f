"""Failure detection, elastic recovery and fault injection for multi-process runs.

Reference: rollout workers are wrapped in a ``BackoffSupervisor``
and death-watched by the router; a ``Terminated`` child is replaced
(`TrainerRouterActor.scala:46-64,101-102,116-120,141-146`) and, in the trained
state, ``StartTraining`` is re-broadcast.  Across processes the same duties are:

* **detect** — every rank publishes a heartbeat into the rendezvous store; a
  :class:`Watchdog` thread flags peers whose heartbeat goes stale (RCCL
  collectives just hang on a dead peer, so a timeout is the only signal), and the
  launcher sees a worker's exit status / signal;
* **replace** — :class:`ElasticRunner` tears the whole generation down (a
  communicator with a dead member cannot be repaired), re-rendezvouses on a
  fresh port with generation ``g+1`` and respawns every rank (backoff between
  attempts, like the reference's 3 s .. 1 min backoff supervisor);
* **re-dispatch** — workers resume from the newest checkpoint written by rank 0
  (deterministic C++ writer) and rank 0's weights/optimizer state are broadcast,
  the analogue of re-sending ``Train`` to the replacement routee;
* **inject** — ``SHARETRADE_FAIL_AT="rank:step[:generation]"`` makes a worker
  die at a given step (``os._exit``), :func:`kill_worker` SIGKILLs a pid.
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
def fail_point(rank: int, step: int, generation: int = 0) -> None:
    """Die abruptly if ``SHARETRADE_FAIL_AT`` names this rank/step (and generation)."""
    spec = os.environ.get("SHARETRADE_FAIL_AT", "")
    if not spec:
        return
    parts = [int(x) for x in spec.split(":")]
    r, s = parts[0], parts[1]
    g = parts[2] if len(parts) > 2 else 0
    if r == rank and s == step and g == generation:
        os._exit(17)


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
    """Flags peers whose heartbeat is older than ``timeout_s`` (calls ``on_dead(rank)``)."""

    def __init__(self, store, world_size: int, generation: int = 0, timeout_s: float = 5.0,
                 on_dead: Optional[Callable[[int], None]] = None, poll_s: float = 0.5):
        self.store, self.world, self.gen = store, world_size, generation
        self.timeout, self.poll = timeout_s, poll_s
        self.on_dead = on_dead
        self.dead: List[int] = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, name="watchdog", daemon=True)

    def check(self) -> List[int]:
        now = time.time()
        dead = []
        for r in range(self.world):
            try:
                t = float(self.store.get(f"hb/{self.gen}/{r}").decode())
            except Exception:  # noqa: BLE001
                continue
            if now - t > self.timeout:
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

    @property
    def restarts(self) -> int:
        return max(0, len(self.generations) - 1)


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
                 env: Optional[Dict[str, str]] = None):
        self.fn, self.world, self.args = fn, world, args
        self.max_restarts = max_restarts
        self.min_b, self.max_b, self.jitter = min_backoff_s, max_backoff_s, jitter
        self.gen_timeout = gen_timeout_s
        self.env = dict(env or {})

    def run(self) -> ElasticResult:
        res = ElasticResult(ok=False)
        ctx = mp.get_context("spawn")
        for gen in range(self.max_restarts + 1):
            if gen:
                time.sleep(calculate_delay(gen - 1, self.min_b, self.max_b, self.jitter))
            port = free_port()
            t0 = time.perf_counter()
            procs = [ctx.Process(target=_entry, args=(r, self.fn, self.world, port, gen, self.args, self.env),
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
                if time.monotonic() > deadline:
                    failed = True
                    break
                time.sleep(0.02)
            if failed:
                # peers are likely blocked in a collective with the dead rank: tear down
                for p in procs:
                    if p.exitcode is None:
                        p.kill()
            for p in procs:
                p.join(timeout=30)
            gr = GenerationResult(gen, {r: p.exitcode for r, p in enumerate(procs)}, not failed,
                                  time.perf_counter() - t0)
            res.generations.append(gr)
            if not failed:
                res.ok = True
                return res
        return res
