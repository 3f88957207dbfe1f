"""Engine-backed rollout workers: the actor API on top of the vectorised data plane.

In the reference every ``TrainerChildActor`` steps its own episode and makes two
blocking asks per step to the shared learner (`TrainerChildActor.scala:82-103`),
so 10 workers = 116,920 serialized mailbox round trips per run.
Here the workers keep their FSM, their messages and their supervision, but
``train`` asks one :class:`EngineActor` to ``RunEpisode``; the engine actor
gathers the requests that arrive together (all ``Train`` broadcasts of one
``StartTraining``) and runs them as lanes of ONE :class:`VectorEngine` — every
step of every worker in one or two kernel launches — then answers each worker
with its own final portfolio.  The learner is shared across the lanes exactly
like the reference's single ``QDecisionPolicyActor``, and its parameters persist
across episodes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import numpy as np
import torch

from ..actors.runtime import Actor, ActorRef, NotHandled, Props, pipe_to, singleton
from ..config import Config
from ..errors import IllegalArgumentException
from .child import TrainerChildActor

_Go = singleton("EngineActor._Go")


@dataclass(frozen=True, eq=False)
class RunEpisode:
    stock_data: Any
    budget: float
    shares: int


@dataclass(frozen=True, eq=False)
class _Done:
    batch: List[Tuple[Optional[ActorRef], RunEpisode]]
    finals: List[float]


@dataclass(frozen=True, eq=False)
class _Failed:
    batch: List[Tuple[Optional[ActorRef], RunEpisode]]
    cause: BaseException


class EngineActor(Actor):
    def __init__(self, cfg: Config, device: Optional[torch.device] = None, gather_window_s: float = 0.05):
        self.cfg = cfg
        self.device = device
        self.window = gather_window_s
        self.pending: List[Tuple[Optional[ActorRef], RunEpisode]] = []
        self.scheduled = False
        self.running = False
        self.params: Optional[torch.Tensor] = None
        self.episodes_run = 0
        self.last_engine_stats = {}

    @classmethod
    def props(cls, cfg: Config, device: Optional[torch.device] = None, **kw) -> Props:
        return Props(cls, cfg, device, **kw)

    def receive(self, msg: Any) -> Any:
        if isinstance(msg, RunEpisode):
            self.pending.append((self.sender, msg))
            self._schedule()
            return None
        if msg is _Go:
            self.scheduled = False
            if self.running or not self.pending:
                return None
            key = self._key(self.pending[0][1])
            batch = [p for p in self.pending if self._key(p[1]) == key]
            self.pending = [p for p in self.pending if self._key(p[1]) != key]
            self.running = True
            fut = self.context.system.blocking_future(lambda: self._run_batch(batch), name="engine")
            pipe_to(fut.map(lambda finals: _Done(batch, finals)).recover(lambda e: _Failed(batch, e)),
                    self.self_ref)
            return None
        if isinstance(msg, _Done):
            self.running = False
            for (snd, _), fin in zip(msg.batch, msg.finals):
                if snd is not None:
                    snd.tell(float(fin), self.self_ref)
            if self.pending:
                self._schedule()
            return None
        if isinstance(msg, _Failed):
            self.running = False
            from ..actors.runtime import Status

            for snd, _ in msg.batch:
                if snd is not None:
                    snd.tell(Status.Failure(msg.cause), self.self_ref)
            if self.pending:
                self._schedule()
            return None
        return NotHandled

    @staticmethod
    def _key(r: RunEpisode):
        return (id(r.stock_data), r.budget, r.shares)

    def _schedule(self) -> None:
        if not self.scheduled:
            self.scheduled = True
            self.context.system.scheduler.tell_once(self.window, self.self_ref, _Go)

    # ------------------------------------------------------------------ the data plane
    def _run_batch(self, batch: List[Tuple[Optional[ActorRef], RunEpisode]]) -> List[float]:
        from .engine import VectorEngine

        req = batch[0][1]
        cfg = self.cfg.clone()
        cfg.env.budget = float(req.budget)
        cfg.env.shares = int(req.shares)
        prices = np.asarray(list(req.stock_data.share_prices.values()), dtype=np.float32)
        n = len(batch)
        dev = self.device if self.device is not None else torch.device("cpu")
        E = n
        if dev.type == "cuda" and cfg.engine.dtype == "bf16":
            E = (n + 31) // 32 * 32          # fused kernel works on 32-env chunks; extra lanes are discarded
        bank = torch.from_numpy(prices)[None, :].expand(E, -1).contiguous()
        eng = VectorEngine(cfg, prices=bank, device=dev, envs=E, params=self.params)
        steps = eng.T - eng.H
        eng.run(steps)
        eng.synchronize()
        self.params = eng.params.detach().clone()
        self.episodes_run += 1
        self.last_engine_stats = eng.stats_dict()
        finals = eng.final_portfolios().double().cpu().numpy()[:n]
        if np.isnan(finals).any():
            raise ArithmeticError("episode did not complete")
        return [float(x) for x in finals]


class EngineTrainerChild(TrainerChildActor):
    """A ``TrainerChildActor`` whose episode runs as a lane of the shared engine."""

    def __init__(self, engine: ActorRef, my_budget: float, no_of_stocks: int, cfg: Optional[Config] = None,
                 timeout_s: float = 3600.0):
        super().__init__(engine, my_budget, no_of_stocks, cfg)
        self.engine = engine
        self.timeout_s = timeout_s

    def train(self, stock_data):
        n = len(stock_data.share_prices)
        if n <= self.cfg.model.history:
            raise IllegalArgumentException("Stock price count should be more than Tensorflow input nodes")
        return self.engine.ask(RunEpisode(stock_data, self.my_budget, self.no_of_stocks), self.timeout_s)


def engine_child_props(engine: ActorRef, cfg: Config) -> Props:
    return Props(EngineTrainerChild, engine, cfg.env.budget, cfg.env.shares, cfg)
