"""Routers (``akka.routing``): immutable :class:`Router` + routing logics.

The reference builds ``Router(BroadcastRoutingLogic(), children)`` and
replaces it functionally with ``removeRoutee`` / ``addRoutee`` as workers
finish or die (`TrainerRouterActor.scala:60-66,103-105,141-146`), and answers
``akka.routing.GetRoutees`` with the current routee list (`:132-135`).
"""
from __future__ import annotations

import itertools
import random
import threading
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence, Tuple

from .runtime import ActorRef, singleton

GetRoutees = singleton("GetRoutees")


@dataclass(frozen=True)
class Routees:
    routees: Tuple["ActorRefRoutee", ...]

    def __len__(self) -> int:
        return len(self.routees)

    def __iter__(self):
        return iter(self.routees)

    def __getitem__(self, i):
        return self.routees[i]

    @property
    def size(self) -> int:
        return len(self.routees)


@dataclass(frozen=True)
class ActorRefRoutee:
    ref: ActorRef

    def send(self, msg: Any, sender: Optional[ActorRef] = None) -> None:
        self.ref.tell(msg, sender)


class RoutingLogic:
    def select(self, msg: Any, routees: Sequence[ActorRefRoutee]) -> List[ActorRefRoutee]:
        raise NotImplementedError


class BroadcastRoutingLogic(RoutingLogic):
    def select(self, msg, routees):
        return list(routees)


class RoundRobinRoutingLogic(RoutingLogic):
    def __init__(self):
        self._n = itertools.count()
        self._lock = threading.Lock()

    def select(self, msg, routees):
        if not routees:
            return []
        with self._lock:
            i = next(self._n)
        return [routees[i % len(routees)]]


class RandomRoutingLogic(RoutingLogic):
    def __init__(self, seed: Optional[int] = None):
        self._rng = random.Random(seed)

    def select(self, msg, routees):
        return [self._rng.choice(list(routees))] if routees else []


class Router:
    """Immutable router; ``route`` sends through the logic."""

    def __init__(self, logic: RoutingLogic, routees: Sequence[Any] = ()):
        self.logic = logic
        self.routees: Tuple[ActorRefRoutee, ...] = tuple(
            r if isinstance(r, ActorRefRoutee) else ActorRefRoutee(r) for r in routees)

    def route(self, msg: Any, sender: Optional[ActorRef] = None) -> None:
        for r in self.logic.select(msg, self.routees):
            r.send(msg, sender)

    def add_routee(self, r: Any) -> "Router":
        rr = r if isinstance(r, ActorRefRoutee) else ActorRefRoutee(r)
        return Router(self.logic, self.routees + (rr,))

    def remove_routee(self, r: Any) -> "Router":
        ref = r.ref if isinstance(r, ActorRefRoutee) else r
        return Router(self.logic, tuple(x for x in self.routees if x.ref != ref))

    def with_routees(self, routees: Sequence[Any]) -> "Router":
        return Router(self.logic, routees)

    def get_routees(self) -> Routees:
        return Routees(self.routees)
