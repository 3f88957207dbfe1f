"""Actor API over the multi-process data plane (``python -m sharetrade train --engine vector --gpus N``).

`TrainerRouterActor.scala` fans ``Train`` out to its workers, death-watches them, replaces a dead one
and re-sends it ``Train``, and reduces the workers' final portfolios for ``GetAvg`` / ``GetStd``.  Here:

* every routee is a :class:`RankRoutee` -- a ``TrainerChildActor`` (same FSM, messages, backoff
  supervision) whose ``train`` asks the :class:`RankGroupActor` to run its rank's slice of the episode;
* the :class:`RankGroupActor` binds routees to rank slots, starts the episode on the
  :class:`~sharetrade.parallel.rankgroup.RankGroup` once every rank's routee has asked (the broadcast of
  one ``StartTraining``), and answers each routee with its rank's mean final portfolio;
* a rank's death (exit status or stalled progress) is reported to the actor, which stops that rank's
  routee: the router sees ``Terminated``, creates a replacement and re-sends it ``Train``
  (`TrainerRouterActor.scala:101-102,116-120,141-146`); the replacement takes over the dead routee's
  rank slot while the group respawns its generation and resumes from the last committed shard;
* :class:`DPRouterActor` answers ``GetAvg`` / ``GetStd`` with the statistics the ranks reduced over ALL
  envs of all ranks (``global_mean_std``), ``IsEverythingDone`` from the routees' ``Trained``
  (each rank reports after the ranks' ``all_done``).
"""
from __future__ import annotations

import os
import tempfile
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import numpy as np

from ..actors.future import Future
from ..actors.runtime import Actor, ActorRef, NotHandled, PoisonPill, Props, Status, pipe_to, singleton
from ..config import Config
from ..errors import IllegalArgumentException
from ..parallel.rankgroup import EpisodeResult, RankDeath, RankGroup
from ..protocol import GetAvg, GetStd
from .child import TrainerChildActor
from .router import TrainerRouterActor

GetGlobalStats = singleton("RankGroupActor.GetGlobalStats")
GetDPInfo = singleton("RankGroupActor.GetDPInfo")


@dataclass(frozen=True, eq=False)
class RunRankEpisode:
    stock_data: Any
    routee: ActorRef


@dataclass(frozen=True, eq=False)
class _RankDied:
    death: RankDeath


@dataclass(frozen=True, eq=False)
class _EpisodeDone:
    result: EpisodeResult


@dataclass(frozen=True, eq=False)
class _EpisodeFailed:
    cause: BaseException


class RankGroupActor(Actor):
    """Owns the rank processes; one episode at a time over all ranks."""

    def __init__(self, cfg: Config, world: int, device: str = "cpu", backend: Optional[str] = None,
                 envs_per_rank: int = 10, ckpt_dir: Optional[str] = None, ckpt_every: int = 0,
                 same_device: bool = False, out_dir: Optional[str] = None, group_kw: Optional[Dict] = None):
        self.cfg = cfg
        self.world = int(world)
        self.envs = int(envs_per_rank)
        self.ckpt_root = ckpt_dir or tempfile.mkdtemp(prefix="sharetrade-dp-")
        self.ckpt_every = int(ckpt_every)
        self.out_dir = out_dir
        self.group = RankGroup(self.world, cfg.to_dict(), device=device, backend=backend, same_device=same_device,
                               on_death=self._on_death, **(group_kw or {}))
        self.slots: List[Optional[ActorRef]] = [None] * self.world      # rank -> routee
        self.pending: Dict[int, ActorRef] = {}                          # rank -> asker awaiting the portfolio
        self.results: Optional[EpisodeResult] = None
        self.running = False
        self.episodes = 0
        self.deaths: List[RankDeath] = []
        self.data = None

    @classmethod
    def props(cls, cfg: Config, world: int, **kw) -> Props:
        return Props(cls, cfg, world, **kw)

    def _on_death(self, death: RankDeath) -> None:      # called on the episode's worker thread
        self.self_ref.tell(_RankDied(death), None)

    def post_stop(self) -> None:
        self.group.close()

    def _slot_of(self, routee: ActorRef) -> int:
        for r, s in enumerate(self.slots):
            if s == routee:
                return r
        for r, s in enumerate(self.slots):
            if s is None:
                self.slots[r] = routee
                return r
        raise IllegalArgumentException(f"more routees than ranks ({self.world})")

    def receive(self, msg: Any) -> Any:
        if isinstance(msg, RunRankEpisode):
            r = self._slot_of(msg.routee)
            self.pending[r] = self.sender
            self.data = msg.stock_data
            if self.results is not None and not self.running:
                self._reply(r)
            elif not self.running and len(self.pending) == self.world:
                self._start()
            return None
        if isinstance(msg, _RankDied):
            self.deaths.append(msg.death)
            dead = [msg.death.rank] if msg.death.rank >= 0 else list(range(self.world))
            for r in dead:
                ref = self.slots[r]
                self.slots[r] = None
                self.pending.pop(r, None)
                if ref is not None:
                    self.log.info(f"rank {r} died (generation {msg.death.generation}: {msg.death.reason}); "
                                  f"stopping its routee")
                    ref.tell(PoisonPill, self.self_ref)
            return None
        if isinstance(msg, _EpisodeDone):
            self.running = False
            self.results = msg.result
            self.episodes += 1
            for r in list(self.pending):
                self._reply(r)
            return None
        if isinstance(msg, _EpisodeFailed):
            self.running = False
            for r, asker in list(self.pending.items()):
                asker.tell(Status.Failure(msg.cause), self.self_ref)
            self.pending.clear()
            return None
        if msg is GetDPInfo:
            res = self.results
            self.sender.tell({"world": self.world, "episodes": self.episodes,
                              "deaths": [(d.generation, d.rank, d.reason) for d in self.deaths],
                              "generation": self.group.gen,
                              "ranks": list(res.ranks) if res is not None else None,
                              "global": res.global_stats if res is not None else None}, self.self_ref)
            return None
        if msg is GetGlobalStats:
            self.sender.tell(self.results.global_stats if self.results is not None else None, self.self_ref)
            return None
        return NotHandled

    def _reply(self, r: int) -> None:
        asker = self.pending.pop(r, None)
        if asker is not None:
            asker.tell(float(self.results.ranks[r]["rank_mean"]), self.self_ref)

    def _start(self) -> None:
        prices = np.asarray(list(self.data.share_prices.values()), dtype=np.float32)
        ep = os.path.join(self.ckpt_root, f"episode-{self.episodes}")
        self.running = True
        self.results = None

        def work():
            return self.group.run_episode(prices, self.envs, ep, self.ckpt_every, out_dir=self.out_dir)

        fut = self.context.system.blocking_future(work, name="rank-episode")
        pipe_to(fut.map(_EpisodeDone).recover(_EpisodeFailed), self.self_ref)


class RankRoutee(TrainerChildActor):
    """A rollout worker whose episode is its rank's slice of the data-parallel episode."""

    def __init__(self, group: ActorRef, my_budget: float, no_of_stocks: int, cfg: Optional[Config] = None,
                 timeout_s: float = 24 * 3600.0):
        super().__init__(group, my_budget, no_of_stocks, cfg)
        self.group = group
        self.timeout_s = timeout_s

    def train(self, stock_data) -> Future:
        if len(stock_data.share_prices) <= self.cfg.model.history:
            raise IllegalArgumentException("Stock price count should be more than Tensorflow input nodes")
        return self.group.ask(RunRankEpisode(stock_data, self.self_ref), self.timeout_s)


class DPRouterActor(TrainerRouterActor):
    """``TrainerRouterActor`` whose ``GetAvg`` / ``GetStd`` come from the ranks' all-env reduction."""

    def __init__(self, group: ActorRef, *args, **kw):
        self.group = group
        super().__init__(*args, **kw)

    def _common(self, msg: Any, data, actors, router) -> bool:
        if (msg is GetAvg or msg is GetStd) and actors is not None:
            key = "mean" if msg is GetAvg else "std"
            fut = self.group.ask(GetGlobalStats, self.cfg.router.ask_timeout_s).map(
                lambda st: self._reply_value(float(st[key])) if st is not None else self._reply_value(float("nan")))
            pipe_to(fut, self.sender)
            return True
        return super()._common(msg, data, actors, router)


def rank_routee_props(group: ActorRef, cfg: Config) -> Props:
    return Props(RankRoutee, group, cfg.env.budget, cfg.env.shares, cfg)
