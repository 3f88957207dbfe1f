"""Finite-state-machine actors (``akka.actor.FSM``).

The rollout worker of the reference is ``FSM[TrainerState, TrainerData]``
(`TrainerChildActor.scala:26-62`): ``startWith(Ready, NotComputed)``,
``when(Ready) { case Event(msg, data) => ... stay() / goto(S) using d }``,
``initialize()``.  Subclasses here declare handlers with :meth:`FSM.when` and
return :meth:`stay` / :meth:`goto` (optionally ``.using(data)``) from them.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional

from .runtime import Actor, NotHandled


@dataclass
class Event:
    """``Event(msg, stateData)`` as passed to a state handler."""

    msg: Any
    data: Any


class _Transition:
    __slots__ = ("state", "data", "replies")

    def __init__(self, state: Any, data: Any):
        self.state = state
        self.data = data
        self.replies: List[Any] = []

    def using(self, data: Any) -> "_Transition":
        self.data = data
        return self

    def replying(self, msg: Any) -> "_Transition":
        self.replies.append(msg)
        return self


_KEEP = object()


@dataclass(frozen=True)
class CurrentState:
    fsm: Any
    state: Any


@dataclass(frozen=True)
class Transition:
    fsm: Any
    from_state: Any
    to_state: Any


class FSM(Actor):
    """Base FSM actor.  Handlers: ``fn(event) -> _Transition | NotHandled``."""

    def __init__(self):
        self._handlers: Dict[Any, Callable[[Event], Any]] = {}
        self._unhandled_handler: Optional[Callable[[Event], Any]] = None
        self._transition_hooks: List[Callable[[Any, Any], None]] = []
        self.state_name: Any = None
        self.state_data: Any = None

    # ------------------------------------------------------------ DSL
    def start_with(self, state: Any, data: Any) -> None:
        self.state_name, self.state_data = state, data

    def when(self, state: Any, handler: Callable[[Event], Any]) -> None:
        self._handlers[state] = handler

    def when_unhandled(self, handler: Callable[[Event], Any]) -> None:
        self._unhandled_handler = handler

    def on_transition(self, hook: Callable[[Any, Any], None]) -> None:
        self._transition_hooks.append(hook)

    def initialize(self) -> None:
        if self.state_name is None:
            raise RuntimeError("FSM.initialize() before start_with()")

    def stay(self) -> _Transition:
        return _Transition(self.state_name, self.state_data)

    def goto(self, state: Any) -> _Transition:
        if state not in self._handlers:
            raise KeyError(f"next state {state!r} does not exist")
        return _Transition(state, self.state_data)

    def stop_fsm(self) -> _Transition:
        self.context.stop(self.self_ref)
        return self.stay()

    # ------------------------------------------------------------ dispatch
    def receive(self, msg: Any) -> Any:
        ev = Event(msg, self.state_data)
        h = self._handlers.get(self.state_name)
        r = h(ev) if h is not None else NotHandled
        if r is NotHandled and self._unhandled_handler is not None:
            r = self._unhandled_handler(ev)
        if r is NotHandled or r is None:
            self.log.warning(f"unhandled event {msg!r} in state {self.state_name!r}")
            return None
        self._apply(r)
        return None

    def _apply(self, t: _Transition) -> None:
        old = self.state_name
        self.state_name, self.state_data = t.state, t.data
        for m in t.replies:
            if self.sender is not None:
                self.sender.tell(m, self.self_ref)
        if old != t.state:
            for hook in self._transition_hooks:
                hook(old, t.state)
