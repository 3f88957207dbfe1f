"""Composable futures for the actor control plane.

The reference composes ``scala.concurrent.Future`` everywhere: ``ask`` returns
one, ``pipeTo`` forwards its outcome as a message, and the rollout fold chains
them (`TrainerChildActor.scala:82-103`, `TrainerRouterActor.scala:89-94,137-139`,
`SharePriceGetter.scala:32-36`).  :class:`Future` here is a small promise with
``map`` / ``flat_map`` / ``recover`` / ``on_complete`` and :func:`sequence`,
callbacks run on the caller-supplied executor (the actor system's dispatcher)
or inline.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Iterable, List, Optional


class AskTimeoutException(TimeoutError):
    """An ``ask`` got no reply in time (akka.pattern.AskTimeoutException)."""


class _Inline:
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn

    def __call__(self, f):
        self.fn(f)


class Future:
    __slots__ = ("_cond", "_done", "_value", "_exc", "_callbacks", "_executor")

    def __init__(self, executor: Optional[Callable[[Callable[[], None]], None]] = None):
        self._cond = threading.Condition()
        self._done = False
        self._value: Any = None
        self._exc: Optional[BaseException] = None
        self._callbacks: List[Callable[["Future"], None]] = []
        self._executor = executor

    # ------------------------------------------------------------ completion
    @classmethod
    def successful(cls, value: Any) -> "Future":
        f = cls()
        f.set_result(value)
        return f

    @classmethod
    def failed(cls, exc: BaseException) -> "Future":
        f = cls()
        f.set_exception(exc)
        return f

    def _complete(self, value: Any, exc: Optional[BaseException]) -> bool:
        with self._cond:
            if self._done:
                return False
            self._value, self._exc, self._done = value, exc, True
            cbs, self._callbacks = self._callbacks, []
            self._cond.notify_all()
        for cb in cbs:
            self._run(cb)
        return True

    def set_result(self, value: Any) -> bool:
        return self._complete(value, None)

    def set_exception(self, exc: BaseException) -> bool:
        return self._complete(None, exc)

    def _run(self, cb: Callable[["Future"], None]) -> None:
        if self._executor is not None and not isinstance(cb, _Inline):
            self._executor(lambda: cb(self))
        else:
            cb(self)

    # ------------------------------------------------------------ inspection
    def done(self) -> bool:
        return self._done

    @property
    def is_completed(self) -> bool:
        return self._done

    def result(self, timeout: Optional[float] = None) -> Any:
        with self._cond:
            if not self._done:
                self._cond.wait(timeout)
            if not self._done:
                raise AskTimeoutException(f"future not completed within {timeout}s")
        if self._exc is not None:
            raise self._exc
        return self._value

    def exception(self, timeout: Optional[float] = None) -> Optional[BaseException]:
        with self._cond:
            if not self._done:
                self._cond.wait(timeout)
        return self._exc

    def value(self):
        """``None`` while pending, else ``("ok", v)`` or ``("err", exc)``."""
        if not self._done:
            return None
        return ("err", self._exc) if self._exc is not None else ("ok", self._value)

    # ------------------------------------------------------------ combinators
    def on_complete(self, cb: Callable[["Future"], None], inline: bool = False) -> None:
        """``cb(self)`` once completed, on the executor -- or ``inline`` on the completing thread (for
        trivial, thread-safe callbacks such as cancelling a timer: no dispatcher hop)."""
        if inline:
            cb = _Inline(cb)
        with self._cond:
            if not self._done:
                self._callbacks.append(cb)
                return
        self._run(cb)

    def map(self, fn: Callable[[Any], Any]) -> "Future":
        out = Future(self._executor)

        def cb(f: "Future"):
            if f._exc is not None:
                out.set_exception(f._exc)
                return
            try:
                out.set_result(fn(f._value))
            except BaseException as e:  # noqa: BLE001 - propagate into the future
                out.set_exception(e)

        self.on_complete(cb)
        return out

    def flat_map(self, fn: Callable[[Any], "Future"]) -> "Future":
        out = Future(self._executor)

        def cb(f: "Future"):
            if f._exc is not None:
                out.set_exception(f._exc)
                return
            try:
                nxt = fn(f._value)
            except BaseException as e:  # noqa: BLE001
                out.set_exception(e)
                return
            nxt.on_complete(lambda g: out._complete(g._value, g._exc))

        self.on_complete(cb)
        return out

    def recover(self, fn: Callable[[BaseException], Any]) -> "Future":
        out = Future(self._executor)

        def cb(f: "Future"):
            if f._exc is None:
                out.set_result(f._value)
                return
            try:
                out.set_result(fn(f._exc))
            except BaseException as e:  # noqa: BLE001
                out.set_exception(e)

        self.on_complete(cb)
        return out

    def map_to(self, *types) -> "Future":
        """``mapTo[T]``: fail with ``TypeError`` (ClassCastException) on a mismatch."""
        def check(v):
            if types and not isinstance(v, types):
                raise TypeError(f"cannot cast {type(v).__name__} to {'|'.join(t.__name__ for t in types)}")
            return v
        return self.map(check)


def sequence(futures: Iterable[Future], executor=None) -> Future:
    """``Future.sequence``: all values in order, or the first failure."""
    futs = list(futures)
    out = Future(executor)
    if not futs:
        out.set_result([])
        return out
    results: List[Any] = [None] * len(futs)
    remaining = [len(futs)]
    lock = threading.Lock()

    def make_cb(i):
        def cb(f: Future):
            if f._exc is not None:
                out.set_exception(f._exc)
                return
            results[i] = f._value
            with lock:
                remaining[0] -= 1
                last = remaining[0] == 0
            if last:
                out.set_result(list(results))
        return cb

    for i, f in enumerate(futs):
        f.on_complete(make_cb(i))
    return out
