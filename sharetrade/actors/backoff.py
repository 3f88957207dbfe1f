"""Backoff supervision (``akka.pattern.BackoffSupervisor`` with ``Backoff.onFailure``).

The reference wraps every rollout worker (`TrainerRouterActor.scala:46-58`)::

    BackoffSupervisor.props(Backoff.onFailure(childTrainerProp, "child-trainer",
        3 seconds, 1 minute, 0.2).withSupervisorStrategy(OneForOneStrategy() {
          case _: ArithmeticException      => Resume
          case _: NullPointerException     => Restart
          case _: IllegalArgumentException => Stop
          case _: Exception                => Escalate }))

Semantics reproduced (Akka 2.5 ``BackoffOnRestartSupervisor``):

* the wrapper creates the child under ``child_name`` and watches it;
* messages from the child go to the wrapper's parent *with the wrapper as
  sender*; every other message is forwarded to the child (dead letters when
  there is none);
* a failure the strategy maps to **Restart** stops the child and re-creates it
  after ``min(max_backoff, min_backoff * 2**n) * (1 + U[0, random_factor))``,
  ``n`` = restarts so far; the count resets once a child has lived
  ``reset_after`` seconds (AutoReset(minBackoff));
* **Resume** resumes the child, **Escalate** fails the wrapper;
* if the child stops (Stop directive, PoisonPill, ...) the wrapper stops too,
  so the router's death watch on the wrapper fires.
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Any, Optional

from .runtime import (Actor, ActorRef, Directive, Escalate, Props, Restart, Resume, Stop, SupervisorStrategy,
                      Terminated, singleton)

StartChild = singleton("BackoffSupervisor.StartChild")
GetCurrentChild = singleton("BackoffSupervisor.GetCurrentChild")
GetRestartCount = singleton("BackoffSupervisor.GetRestartCount")
Reset = singleton("BackoffSupervisor.Reset")


@dataclass(frozen=True)
class CurrentChild:
    ref: Optional[ActorRef]


@dataclass(frozen=True)
class RestartCount:
    count: int


@dataclass(frozen=True)
class _ResetRestartCount:
    current: int


def calculate_delay(restart_count: int, min_backoff: float, max_backoff: float, random_factor: float,
                    rng: Optional[random.Random] = None) -> float:
    """``BackoffSupervisor.calculateDelay``."""
    r = (rng or random).random()
    rnd = 1.0 + r * random_factor
    if restart_count >= 30:
        return max_backoff
    return min(max_backoff, min_backoff * (2.0 ** restart_count)) * rnd


@dataclass
class BackoffOptions:
    child_props: Props
    child_name: str
    min_backoff_s: float
    max_backoff_s: float
    random_factor: float
    strategy: Optional[SupervisorStrategy] = None
    reset_after_s: Optional[float] = None   # default AutoReset(minBackoff)

    def with_supervisor_strategy(self, strategy: SupervisorStrategy) -> "BackoffOptions":
        self.strategy = strategy
        return self


class Backoff:
    @staticmethod
    def on_failure(child_props: Props, child_name: str, min_backoff_s: float, max_backoff_s: float,
                   random_factor: float) -> BackoffOptions:
        return BackoffOptions(child_props, child_name, min_backoff_s, max_backoff_s, random_factor)


class _BackoffStrategy(SupervisorStrategy):
    def __init__(self, owner: "BackoffSupervisor", user: SupervisorStrategy):
        super().__init__(None, user.one_for_one)
        self.owner, self.user = owner, user

    def decide(self, exc: BaseException) -> str:
        d = self.user.decide(exc)
        if d == Restart:
            self.owner._restart_child_with_backoff()
            return Directive.Handled
        return d


class BackoffSupervisor(Actor):
    def __init__(self, opts: BackoffOptions, seed: Optional[int] = None):
        self.opts = opts
        self.child: Optional[ActorRef] = None
        self.restart_count = 0
        self._waiting_for: Optional[ActorRef] = None
        self._rng = random.Random(seed)
        self.supervisor_strategy = _BackoffStrategy(self, opts.strategy or SupervisorStrategy())

    @classmethod
    def props(cls, opts: BackoffOptions, seed: Optional[int] = None) -> Props:
        return Props(cls, opts, seed)

    def pre_start(self) -> None:
        self._start_child()

    def _start_child(self) -> None:
        if self.child is None:
            self.child = self.context.watch(self.context.actor_of(self.opts.child_props, self.opts.child_name))
            reset = self.opts.reset_after_s if self.opts.reset_after_s is not None else self.opts.min_backoff_s
            self.context.system.scheduler.tell_once(reset, self.self_ref, _ResetRestartCount(self.restart_count))

    def _restart_child_with_backoff(self) -> None:
        c = self.child
        if c is None:
            return
        self._waiting_for = c
        self.context.stop(c)

    def receive(self, msg: Any) -> Any:
        if isinstance(msg, Terminated):
            if self._waiting_for is not None and msg.actor == self._waiting_for:
                self._waiting_for = None
                self.child = None
                delay = calculate_delay(self.restart_count, self.opts.min_backoff_s, self.opts.max_backoff_s,
                                        self.opts.random_factor, self._rng)
                self.restart_count += 1
                self.context.system.scheduler.tell_once(delay, self.self_ref, StartChild)
                return None
            if self.child is not None and msg.actor == self.child:
                self.log.debug(f"Terminating, because child [{msg.actor}] terminated itself")
                self.child = None
                self.context.stop(self.self_ref)
                return None
            return None
        if msg is StartChild:
            self._start_child()
            return None
        if isinstance(msg, _ResetRestartCount):
            if msg.current == self.restart_count:
                self.restart_count = 0
            return None
        if msg is Reset:
            self.restart_count = 0
            return None
        if msg is GetRestartCount:
            self.sender.tell(RestartCount(self.restart_count), self.self_ref)
            return None
        if msg is GetCurrentChild:
            self.sender.tell(CurrentChild(self.child), self.self_ref)
            return None
        if self.child is not None and self.sender is not None and self.sender == self.child:
            # use the BackoffSupervisor as sender
            parent = self.context.parent
            if parent is not None:
                parent.tell(msg, self.self_ref)
            return None
        if self.child is not None:
            self.child.tell(msg, self.sender)
        else:
            self.context.system.dead_letters.tell(msg, self.sender)
        return None


__all__ = ["Backoff", "BackoffOptions", "BackoffSupervisor", "calculate_delay", "StartChild", "GetCurrentChild",
           "GetRestartCount", "CurrentChild", "RestartCount", "Reset", "Resume", "Restart", "Stop", "Escalate"]
