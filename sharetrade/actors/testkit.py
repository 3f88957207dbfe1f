"""TestKit for the actor runtime (``akka.testkit``).

Mirrors what the reference's specs use (`src/test/scala/*.scala`):
``TestProbe`` (fake learner / fake parent), ``ImplicitSender``-style
``TestKit.send``, ``expect_msg`` / ``expect_msg_type`` / ``expect_no_message``,
``reply``, ``await_assert``, ``TestActorRef(props, parent, name)`` and
``EventFilter[Exception](occurrences=n).intercept``.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from contextlib import contextmanager
from typing import Any, Callable, List, Optional, Tuple, Type

from .runtime import Actor, ActorRef, ActorSystem, LogEvent, Props

DEFAULT_TIMEOUT = 3.0          # akka.test.single-expect-default
NO_MSG_DEFAULT = 0.1           # expectNoMessage() default (akka.test.expect-no-message-default)


class _ProbeActor(Actor):
    def __init__(self, q: "queue.Queue[Tuple[Any, Optional[ActorRef]]]", auto: List[Callable]):
        self.q = q
        self.auto = auto

    def receive(self, msg: Any) -> Any:
        for fn in list(self.auto):
            r = fn(msg, self.sender)
            if r:
                return None
        self.q.put((msg, self.sender))
        return None


class TestProbe:
    __test__ = False  # not a pytest class

    def __init__(self, system: ActorSystem, name: Optional[str] = None):
        self.system = system
        self._q: "queue.Queue[Tuple[Any, Optional[ActorRef]]]" = queue.Queue()
        self._auto: List[Callable] = []
        self.ref = system.actor_of(Props(_ProbeActor, self._q, self._auto), name)
        self.last_sender: Optional[ActorRef] = None
        self.last_message: Any = None

    # ------------------------------------------------------------ sending
    def send(self, target: ActorRef, msg: Any) -> None:
        target.tell(msg, self.ref)

    def reply(self, msg: Any) -> None:
        if self.last_sender is None:
            raise AssertionError("reply(): no last sender")
        self.last_sender.tell(msg, self.ref)

    def forward(self, target: ActorRef, msg: Any = None) -> None:
        target.tell(self.last_message if msg is None else msg, self.last_sender)

    def set_auto_pilot(self, fn: Callable[[Any, Optional[ActorRef]], bool]) -> None:
        """``fn(msg, sender) -> True`` consumes the message (TestActor.AutoPilot)."""
        self._auto.append(fn)

    # ------------------------------------------------------------ expectations
    def receive_one(self, timeout: Optional[float] = DEFAULT_TIMEOUT) -> Any:
        try:
            msg, snd = self._q.get(timeout=timeout)
        except queue.Empty:
            raise AssertionError(f"timeout ({timeout}s) during receive_one while waiting for a message")
        self.last_message, self.last_sender = msg, snd
        return msg

    def expect_msg(self, expected: Any, timeout: float = DEFAULT_TIMEOUT) -> Any:
        msg = self.receive_one(timeout)
        if msg != expected and msg is not expected:
            raise AssertionError(f"expected {expected!r}, found {msg!r}")
        return msg

    def expect_msg_type(self, typ, timeout: float = DEFAULT_TIMEOUT) -> Any:
        msg = self.receive_one(timeout)
        if not isinstance(msg, typ):
            raise AssertionError(f"expected message of type {typ}, found {type(msg).__name__}: {msg!r}")
        return msg

    def expect_msg_pf(self, fn: Callable[[Any], Any], timeout: float = DEFAULT_TIMEOUT) -> Any:
        msg = self.receive_one(timeout)
        return fn(msg)

    def expect_no_message(self, duration: float = NO_MSG_DEFAULT) -> None:
        try:
            msg, snd = self._q.get(timeout=duration)
        except queue.Empty:
            return
        raise AssertionError(f"received unexpected message {msg!r}")

    def receive_n(self, n: int, timeout: float = DEFAULT_TIMEOUT) -> List[Any]:
        deadline = time.monotonic() + timeout
        return [self.receive_one(max(0.0, deadline - time.monotonic())) for _ in range(n)]

    def fish_for_message(self, pred: Callable[[Any], bool], timeout: float = DEFAULT_TIMEOUT) -> Any:
        deadline = time.monotonic() + timeout
        while True:
            msg = self.receive_one(max(0.0, deadline - time.monotonic()))
            if pred(msg):
                return msg

    def watch(self, ref: ActorRef) -> ActorRef:
        return self.ref._cell.context.watch(ref)

    def expect_terminated(self, ref: ActorRef, timeout: float = DEFAULT_TIMEOUT):
        from .runtime import Terminated

        return self.fish_for_message(lambda m: isinstance(m, Terminated) and m.actor == ref, timeout)


class TestKit(TestProbe):
    """A test driver with an implicit sender (``ImplicitSender``): ``kit.tell(ref, msg)``."""

    __test__ = False

    def __init__(self, system: Optional[ActorSystem] = None, name: str = "testActor"):
        self.owns_system = system is None
        super().__init__(system or ActorSystem("TestSystem", loglevel="DEBUG"), name)

    def tell(self, target: ActorRef, msg: Any) -> None:
        target.tell(msg, self.ref)

    def ask(self, target: ActorRef, msg: Any, timeout: float = 10.0):
        return target.ask(msg, timeout)

    def shutdown(self) -> None:
        if self.owns_system:
            self.system.terminate()


def await_assert(fn: Callable[[], Any], max_s: float = DEFAULT_TIMEOUT, interval_s: float = 0.1) -> Any:
    """Retry ``fn`` until it stops raising ``AssertionError`` (``awaitAssert``)."""
    deadline = time.monotonic() + max_s
    while True:
        try:
            return fn()
        except AssertionError:
            if time.monotonic() >= deadline:
                raise
            time.sleep(interval_s)


def await_cond(pred: Callable[[], bool], max_s: float = DEFAULT_TIMEOUT, interval_s: float = 0.05) -> None:
    deadline = time.monotonic() + max_s
    while not pred():
        if time.monotonic() >= deadline:
            raise AssertionError(f"condition not met within {max_s}s")
        time.sleep(interval_s)


def TestActorRef(system: ActorSystem, props: Props, parent: Optional[ActorRef] = None,
                 name: Optional[str] = None) -> ActorRef:
    """Spawn ``props`` as a child of ``parent`` (a probe), so ``context.parent``
    messages land in the probe (`TrainerChildActorSpec.scala:65`)."""
    pcell = parent._cell if parent is not None else None
    return system._spawn(props, name, pcell)


class EventFilter:
    """``EventFilter[T](occurrences = n) intercept { ... }``: wait until exactly
    ``occurrences`` error events whose cause is a ``T`` were logged."""

    def __init__(self, system: ActorSystem, exc_type: Type[BaseException] = Exception, occurrences: int = 1,
                 message: Optional[str] = None, level: int = logging.ERROR, timeout: float = DEFAULT_TIMEOUT):
        self.system = system
        self.exc_type = exc_type
        self.occurrences = occurrences
        self.message = message
        self.level = level
        self.timeout = timeout
        self.matched: List[LogEvent] = []
        self._lock = threading.Lock()

    def _sub(self, ev: Any) -> None:
        if not isinstance(ev, LogEvent) or ev.level < self.level:
            return
        if self.exc_type is not None and not isinstance(ev.cause, self.exc_type):
            return
        if self.message is not None and self.message not in ev.message:
            return
        with self._lock:
            self.matched.append(ev)

    @contextmanager
    def intercept(self):
        self.system.event_stream.subscribe(self._sub)
        try:
            yield self
            await_cond(lambda: len(self.matched) >= self.occurrences, self.timeout)
            time.sleep(0.05)
            if len(self.matched) != self.occurrences:
                raise AssertionError(f"expected {self.occurrences} {self.exc_type.__name__} events, "
                                     f"got {len(self.matched)}")
        finally:
            self.system.event_stream.unsubscribe(self._sub)
