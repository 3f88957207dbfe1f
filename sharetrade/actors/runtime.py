"""Actor runtime — the control plane of the engine.

The reference is built on Akka 2.5 (`build.sbt:10-14`): mailbox actors with
``tell``/``ask``, ``context.become``, ``Stash``, death watch (``watch`` /
``Terminated``), ``PoisonPill``, supervision (`TrainerRouterActor.scala:46-58`)
and a fork-join dispatcher.  This module provides those semantics natively in
Python for the *control plane* only — the data plane (Q-network math, env
steps, gradient sync) runs in HIP kernels and RCCL collectives and never goes
through a mailbox on the hot path.

Semantics kept from Akka:

* one message at a time per actor (an actor is never run by two threads);
  a per-actor FIFO mailbox, system messages (failure, watch, terminate)
  processed before ordinary ones;
* ``sender`` is captured per message, replies go to it; ``forward`` keeps it;
* an exception in ``receive`` suspends the actor and asks the parent's
  :class:`SupervisorStrategy` (Resume / Restart / Stop / Escalate);
  the default strategy restarts on ``Exception``;
* ``stop`` stops children first, then ``post_stop``, then every watcher gets
  ``Terminated(ref)``; messages to a dead actor go to dead letters;
* ``become`` / ``unbecome`` behaviour stack, ``stash`` / ``unstash_all``;
* ``ask`` returns a :class:`~sharetrade.actors.future.Future` completed by the
  first reply (``Status.Failure`` fails it), or an ``AskTimeoutException``.
"""
from __future__ import annotations

import heapq
import itertools
import logging
import os
import threading
import time
import traceback
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Any, Callable, Deque, Dict, List, Optional, Set, Tuple

from .future import AskTimeoutException, Future

log_root = logging.getLogger("sharetrade.actors")


# ====================================================================== messages
class _Singleton:
    _name = "?"

    def __repr__(self) -> str:
        return self._name

    def __reduce__(self):
        return self._name


def singleton(name: str):
    cls = type(name, (_Singleton,), {"_name": name})
    return cls()


PoisonPill = singleton("PoisonPill")
Kill = singleton("Kill")


@dataclass(frozen=True)
class Terminated:
    actor: "ActorRef"


class Status:
    @dataclass(frozen=True)
    class Success:
        value: Any

    @dataclass(frozen=True)
    class Failure:
        cause: BaseException


@dataclass(frozen=True)
class DeadLetter:
    message: Any
    sender: Optional["ActorRef"]
    recipient: "ActorRef"


class ActorKilledException(Exception):
    pass


class ActorInitializationException(Exception):
    pass


class DeathPactException(Exception):
    pass


# system messages (processed before the ordinary mailbox)
@dataclass(frozen=True)
class _Failed:
    child: "ActorRef"
    cause: BaseException


@dataclass(frozen=True)
class _Watch:
    watcher: "ActorRef"


@dataclass(frozen=True)
class _Unwatch:
    watcher: "ActorRef"


@dataclass(frozen=True)
class _ChildTerminated:
    child: "ActorRef"


_Resume = singleton("_Resume")
_Restart = singleton("_Restart")
_Stop = singleton("_Stop")


# ====================================================================== supervision
class Directive:
    Resume = "Resume"
    Restart = "Restart"
    Stop = "Stop"
    Escalate = "Escalate"
    Handled = "Handled"   # the strategy dealt with the failure itself (backoff supervision)


Resume, Restart, Stop, Escalate = Directive.Resume, Directive.Restart, Directive.Stop, Directive.Escalate


class SupervisorStrategy:
    """``OneForOneStrategy`` / ``AllForOneStrategy`` with an exception → directive decider.

    ``decider`` is either a callable ``exc -> directive`` or a list of
    ``(ExceptionType, directive)`` pairs matched in order (like a Scala
    partial function, `TrainerRouterActor.scala:53-58`)."""

    def __init__(self, decider=None, one_for_one: bool = True, max_retries: int = -1,
                 within_s: Optional[float] = None, logging_enabled: bool = True):
        self._decider = decider
        self.one_for_one = one_for_one
        self.max_retries = max_retries
        self.within_s = within_s
        self.logging_enabled = logging_enabled
        self._restarts: Dict[int, List[float]] = {}

    def decide(self, exc: BaseException) -> str:
        d = self._decider
        if d is None:
            return default_decider(exc)
        if callable(d):
            r = d(exc)
            return r if r is not None else Escalate
        for typ, directive in d:
            if isinstance(exc, typ):
                return directive
        return Escalate

    def allow_restart(self, child_id: int) -> bool:
        if self.max_retries < 0:
            return True
        now = time.monotonic()
        hist = self._restarts.setdefault(child_id, [])
        if self.within_s is not None:
            hist[:] = [t for t in hist if now - t <= self.within_s]
        if len(hist) >= self.max_retries:
            return False
        hist.append(now)
        return True


def default_decider(exc: BaseException) -> str:
    """Akka's ``SupervisorStrategy.defaultDecider``."""
    if isinstance(exc, (ActorInitializationException, ActorKilledException, DeathPactException)):
        return Stop
    if isinstance(exc, Exception):
        return Restart
    return Escalate


def OneForOneStrategy(decider=None, max_retries: int = -1, within_s: Optional[float] = None) -> SupervisorStrategy:
    return SupervisorStrategy(decider, True, max_retries, within_s)


def AllForOneStrategy(decider=None, max_retries: int = -1, within_s: Optional[float] = None) -> SupervisorStrategy:
    return SupervisorStrategy(decider, False, max_retries, within_s)


DEFAULT_STRATEGY = SupervisorStrategy()


# ====================================================================== props / refs
class Props:
    """Recipe to (re)create an actor: ``Props(cls, *args, **kw)`` or ``Props.create(factory)``."""

    def __init__(self, cls_or_factory: Callable[..., "Actor"], *args, **kwargs):
        self.factory = cls_or_factory
        self.args = args
        self.kwargs = kwargs

    @classmethod
    def create(cls, factory: Callable[[], "Actor"]) -> "Props":
        return cls(factory)

    def new_actor(self) -> "Actor":
        return self.factory(*self.args, **self.kwargs)

    def __repr__(self) -> str:
        f = getattr(self.factory, "__name__", repr(self.factory))
        return f"Props({f})"


class ActorRef:
    """Location-transparent handle.  ``ref.tell(msg, sender)``; ``ref.ask(msg, timeout)``."""

    __slots__ = ("path", "_cell", "_uid", "__weakref__")
    _uids = itertools.count(1)

    def __init__(self, path: str, cell: Optional["ActorCell"]):
        self.path = path
        self._cell = cell
        self._uid = next(ActorRef._uids)

    @property
    def name(self) -> str:
        return self.path.rsplit("/", 1)[-1]

    @property
    def parent_name(self) -> str:
        parts = self.path.rstrip("/").split("/")
        return parts[-2] if len(parts) >= 2 else ""

    def tell(self, msg: Any, sender: Optional["ActorRef"] = None) -> None:
        c = self._cell
        if c is None:
            return
        c.enqueue(msg, sender)

    def forward(self, msg: Any, context: "ActorContext") -> None:
        self.tell(msg, context.sender)

    def ask(self, msg: Any, timeout: float = 10.0, sender: Optional["ActorRef"] = None) -> Future:
        c = self._cell
        system = c.system if c is not None else None
        if system is None:
            return Future.failed(AskTimeoutException(f"ask to {self.path}: no system"))
        return system._ask(self, msg, timeout)

    def is_terminated(self) -> bool:
        c = self._cell
        return c is None or c.dead

    def __repr__(self) -> str:
        return f"Actor[{self.path}#{self._uid}]"

    def __hash__(self) -> int:
        return self._uid

    def __eq__(self, other) -> bool:
        return isinstance(other, ActorRef) and other._uid == self._uid


class _PromiseRef(ActorRef):
    """Temporary reply target of an ``ask``."""

    __slots__ = ("promise", "system")

    def __init__(self, system: "ActorSystem", path: str, promise: Future):
        super().__init__(path, None)
        self.promise = promise
        self.system = system

    def tell(self, msg: Any, sender: Optional[ActorRef] = None) -> None:
        if isinstance(msg, Status.Failure):
            self.promise.set_exception(msg.cause)
        else:
            self.promise.set_result(msg)

    def is_terminated(self) -> bool:
        return self.promise.done()


class _FunctionRef(ActorRef):
    """Ref that calls a Python function on ``tell`` (dead letters, test hooks)."""

    __slots__ = ("fn",)

    def __init__(self, path: str, fn: Callable[[Any, Optional[ActorRef]], None]):
        super().__init__(path, None)
        self.fn = fn

    def tell(self, msg: Any, sender: Optional[ActorRef] = None) -> None:
        self.fn(msg, sender)

    def is_terminated(self) -> bool:
        return False


# ====================================================================== actor
class Actor:
    """Base class.  Override :meth:`receive` (return ``NotHandled`` / raise for
    unhandled messages is not required: unhandled messages are logged).

    Inside ``receive``: ``self.context``, ``self.sender``, ``self.self_ref``,
    ``self.log``; ``self.context.become(fn)`` swaps the behaviour."""

    context: "ActorContext"
    supervisor_strategy: SupervisorStrategy = DEFAULT_STRATEGY

    def receive(self, msg: Any) -> Any:
        return NotHandled

    # lifecycle hooks
    def pre_start(self) -> None:
        pass

    def post_stop(self) -> None:
        pass

    def pre_restart(self, reason: BaseException, message: Any) -> None:
        for c in list(self.context.children):
            self.context.stop(c)
        self.post_stop()

    def post_restart(self, reason: BaseException) -> None:
        self.pre_start()

    def unhandled(self, msg: Any) -> None:
        if isinstance(msg, Terminated):
            raise DeathPactException(f"{self.context.self_ref} got unhandled {msg}")
        self.context.system.event_stream.publish_unhandled(msg, self.context.self_ref)

    # conveniences
    @property
    def sender(self) -> Optional[ActorRef]:
        return self.context.sender

    @property
    def self_ref(self) -> ActorRef:
        return self.context.self_ref

    @property
    def log(self) -> "ActorLogger":
        return self.context.log


NotHandled = singleton("NotHandled")


class Stash:
    """Mixin marker (the reference's ``with Stash``); stash ops live on the context."""

    def stash(self) -> None:
        self.context.stash()

    def unstash_all(self) -> None:
        self.context.unstash_all()


class ActorLogger:
    """``ActorLogging.log`` — publishes to the system event stream."""

    def __init__(self, system: "ActorSystem", source: str):
        self.system, self.source = system, source

    def _pub(self, level: int, msg: str, exc: Optional[BaseException] = None) -> None:
        self.system.event_stream.publish_log(level, self.source, msg, exc)

    def debug(self, msg: str) -> None:
        self._pub(logging.DEBUG, msg)

    def info(self, msg: str) -> None:
        self._pub(logging.INFO, msg)

    def warning(self, msg: str) -> None:
        self._pub(logging.WARNING, msg)

    def error(self, msg: str, exc: Optional[BaseException] = None) -> None:
        self._pub(logging.ERROR, msg, exc)


# ====================================================================== context / cell
class ActorContext:
    def __init__(self, cell: "ActorCell"):
        self._cell = cell
        self.sender: Optional[ActorRef] = None

    @property
    def self_ref(self) -> ActorRef:
        return self._cell.ref

    def mailbox_size(self) -> int:
        """User messages queued behind the current one (a hint: others may enqueue concurrently)."""
        return len(self._cell.mailbox)

    @property
    def parent(self) -> Optional[ActorRef]:
        p = self._cell.parent
        return p.ref if p is not None else None

    @property
    def system(self) -> "ActorSystem":
        return self._cell.system

    @property
    def children(self) -> List[ActorRef]:
        return [c.ref for c in list(self._cell.children.values())]

    def child(self, name: str) -> Optional[ActorRef]:
        c = self._cell.children.get(name)
        return c.ref if c is not None else None

    @property
    def log(self) -> ActorLogger:
        return self._cell.logger

    @property
    def dispatcher(self):
        return self._cell.system.dispatcher

    def actor_of(self, props: Props, name: Optional[str] = None) -> ActorRef:
        return self._cell.system._spawn(props, name, self._cell)

    def stop(self, ref: ActorRef) -> None:
        self._cell.system.stop(ref)

    def watch(self, ref: ActorRef) -> ActorRef:
        c = ref._cell
        me = self._cell.ref
        if c is None or c.dead:
            self._cell.enqueue(Terminated(ref), ref)
        else:
            c.enqueue_system(_Watch(me))
        self._cell.watching.add(ref)
        return ref

    def unwatch(self, ref: ActorRef) -> ActorRef:
        c = ref._cell
        if c is not None:
            c.enqueue_system(_Unwatch(self._cell.ref))
        self._cell.watching.discard(ref)
        return ref

    def become(self, behavior: Callable[[Any], Any], discard_old: bool = True) -> None:
        st = self._cell.behaviors
        if discard_old and st:
            st[-1] = behavior
        else:
            st.append(behavior)

    def unbecome(self) -> None:
        st = self._cell.behaviors
        if len(st) > 1:
            st.pop()

    def stash(self) -> None:
        self._cell.stash_current()

    def unstash_all(self) -> None:
        self._cell.unstash_all()

    def set_receive_timeout(self, seconds: Optional[float]) -> None:
        self._cell.receive_timeout = seconds

    def assert_on_actor_thread(self) -> None:
        """Race check: actor state may only be touched while the actor is
        processing a message, on the dispatcher thread running it."""
        owner = self._cell.running_thread
        if owner != threading.get_ident():
            raise AssertionError(f"{self._cell.ref.path}: state accessed off the actor thread "
                                 f"(owner={owner}, caller={threading.get_ident()})")


class ActorCell:
    _THROUGHPUT = 16

    def __init__(self, system: "ActorSystem", props: Props, path: str, parent: Optional["ActorCell"]):
        self.system = system
        self.props = props
        self.parent = parent
        self.ref = ActorRef(path, self)
        self.children: Dict[str, "ActorCell"] = {}
        self.mailbox: Deque[Tuple[Any, Optional[ActorRef]]] = deque()
        self.sysbox: Deque[Any] = deque()
        self.lock = threading.Lock()
        self.scheduled = False
        self.suspended = False
        self.dead = False
        self.stopping = False
        self.watchers: Set[ActorRef] = set()
        self.watching: Set[ActorRef] = set()
        self.stashed: Deque[Tuple[Any, Optional[ActorRef]]] = deque()
        self.behaviors: List[Callable[[Any], Any]] = []
        self.context = ActorContext(self)
        self.actor: Optional[Actor] = None
        self.current: Optional[Tuple[Any, Optional[ActorRef]]] = None
        self.logger = ActorLogger(system, path)
        self.receive_timeout: Optional[float] = None
        self.child_counter = itertools.count()
        self.failed_cause: Optional[BaseException] = None
        self.running_thread: Optional[int] = None

    # ------------------------------------------------------------ creation
    def create(self) -> None:
        try:
            a = self.props.new_actor()
            a.context = self.context
            self.actor = a
            self.behaviors = [a.receive]
            a.pre_start()
        except Exception as e:  # noqa: BLE001
            self._fail(ActorInitializationException(f"{self.ref.path}: {e!r}"), None)

    # ------------------------------------------------------------ enqueue / schedule
    def enqueue(self, msg: Any, sender: Optional[ActorRef]) -> None:
        with self.lock:
            if self.dead:
                dead = True
            else:
                dead = False
                self.mailbox.append((msg, sender))
        if dead:
            self.system._dead_letter(msg, sender, self.ref)
            return
        self._schedule()

    def enqueue_system(self, msg: Any) -> None:
        with self.lock:
            if self.dead:
                dead = True
            else:
                dead = False
                self.sysbox.append(msg)
        if dead:
            if isinstance(msg, _Watch):
                msg.watcher.tell(Terminated(self.ref), self.ref)
            return
        self._schedule()

    def _schedule(self) -> None:
        with self.lock:
            if self.scheduled or self.dead:
                return
            if not self.sysbox and (self.suspended or not self.mailbox):
                return
            self.scheduled = True
        self.system._execute(self._run)

    # ------------------------------------------------------------ processing
    def _run(self) -> None:
        me = threading.get_ident()
        if self.system.debug and self.running_thread not in (None, me):
            raise AssertionError(f"{self.ref.path}: mailbox processed by two threads at once")
        self.running_thread = me
        try:
            n = 0
            while n < self._THROUGHPUT:
                with self.lock:
                    if self.dead:
                        break
                    if self.sysbox:
                        smsg = self.sysbox.popleft()
                        item = None
                    elif not self.suspended and self.mailbox:
                        item = self.mailbox.popleft()
                        smsg = None
                    else:
                        break
                if smsg is not None:
                    self._system_message(smsg)
                else:
                    self._invoke(*item)
                n += 1
        finally:
            self.running_thread = None
            with self.lock:
                self.scheduled = False
            self._schedule()

    def _invoke(self, msg: Any, sender: Optional[ActorRef]) -> None:
        if self.actor is None:
            return
        self.context.sender = sender
        self.current = (msg, sender)
        try:
            if msg is PoisonPill:
                self.system.stop(self.ref)
                return
            if msg is Kill:
                raise ActorKilledException("Kill")
            if isinstance(msg, Terminated):
                self.watching.discard(msg.actor)
            beh = self.behaviors[-1]
            r = beh(msg)
            if r is NotHandled:
                self.actor.unhandled(msg)
        except Exception as e:  # noqa: BLE001 - supervision
            self._fail(e, msg)
        finally:
            self.current = None

    def _fail(self, exc: BaseException, msg: Any) -> None:
        self.suspended = True
        self.failed_cause = exc
        self._failed_msg = msg
        self.system.event_stream.publish_log(logging.ERROR, self.ref.path, f"{type(exc).__name__}: {exc}", exc)
        if self.parent is None:
            # user guardian: default strategy for top-level actors (restart on Exception)
            if default_decider(exc) == Restart:
                self.enqueue_system(_Restart)
            else:
                self.system.stop(self.ref)
        else:
            self.parent.enqueue_system(_Failed(self.ref, exc))

    def _system_message(self, m: Any) -> None:
        if isinstance(m, _Failed):
            self._handle_child_failure(m.child, m.cause)
        elif isinstance(m, _Watch):
            if m.watcher != self.ref:
                self.watchers.add(m.watcher)
        elif isinstance(m, _Unwatch):
            self.watchers.discard(m.watcher)
        elif isinstance(m, _ChildTerminated):
            self._child_terminated(m.child)
        elif m is _Resume:
            self.suspended = False
            self.failed_cause = None
        elif m is _Restart:
            self._restart()
        elif m is _Stop:
            self.system._stop_cell(self)

    def _handle_child_failure(self, child: ActorRef, cause: BaseException) -> None:
        cc = child._cell
        if cc is None or cc.dead:
            return
        strat = self.actor.supervisor_strategy if self.actor is not None else DEFAULT_STRATEGY
        d = strat.decide(cause)
        targets = [cc] if strat.one_for_one else list(self.children.values())
        if d == Directive.Handled:
            return
        if d == Resume:
            cc.enqueue_system(_Resume)
        elif d == Restart:
            if not strat.allow_restart(child._uid):
                self.system.stop(child)
                return
            for t in targets:
                t.enqueue_system(_Restart)
        elif d == Stop:
            for t in targets:
                self.system.stop(t.ref)
        else:  # Escalate: fail ourselves with the same cause
            self._fail(cause, None)

    def _restart(self) -> None:
        cause = self.failed_cause or Exception("restart")
        old = self.actor
        try:
            if old is not None:
                old.pre_restart(cause, getattr(self, "_failed_msg", None))
        except Exception:  # noqa: BLE001
            pass
        # the stash is handed back to the mailbox (akka.actor.Stash#preRestart)
        self.unstash_all()
        # like Akka, the new incarnation starts only once the old children are gone
        # (their names stay reserved until then)
        deadline = time.monotonic() + 5.0
        while any(not c.dead for c in list(self.children.values())) and time.monotonic() < deadline:
            time.sleep(0.001)
        for k, c in list(self.children.items()):
            if c.dead:
                del self.children[k]
        try:
            a = self.props.new_actor()
            a.context = self.context
            self.actor = a
            self.behaviors = [a.receive]
            a.post_restart(cause)
        except Exception as e:  # noqa: BLE001
            self.failed_cause = ActorInitializationException(repr(e))
            self.system.stop(self.ref)
            return
        self.suspended = False
        self.failed_cause = None

    def _child_terminated(self, child: ActorRef) -> None:
        for k, v in list(self.children.items()):
            if v.ref == child:
                del self.children[k]
        if self.stopping and not self.children:
            self.system._finish_stop(self)

    # ------------------------------------------------------------ stash
    def stash_current(self) -> None:
        if self.current is None:
            raise RuntimeError("stash() outside of message processing")
        self.stashed.append(self.current)

    def unstash_all(self) -> None:
        with self.lock:
            while self.stashed:
                self.mailbox.appendleft(self.stashed.pop())
        self._schedule()


# ====================================================================== event stream
@dataclass
class LogEvent:
    level: int
    source: str
    message: str
    cause: Optional[BaseException] = None
    ts: float = 0.0


class EventStream:
    """Log / dead-letter / unhandled publication (``akka.event.EventStream``).

    Subscribers are callables ``fn(event)``; the default subscriber forwards
    to Python ``logging`` (the reference's slf4j/logback, `application.conf:2-3`)."""

    def __init__(self, loglevel: int = logging.INFO):
        self.loglevel = loglevel
        self._subs: List[Callable[[Any], None]] = []
        self._lock = threading.Lock()

    def subscribe(self, fn: Callable[[Any], None]) -> None:
        with self._lock:
            self._subs.append(fn)

    def unsubscribe(self, fn: Callable[[Any], None]) -> None:
        with self._lock:
            if fn in self._subs:
                self._subs.remove(fn)

    def publish(self, ev: Any) -> None:
        with self._lock:
            subs = list(self._subs)
        for s in subs:
            try:
                s(ev)
            except Exception:  # noqa: BLE001
                traceback.print_exc()

    def publish_log(self, level: int, source: str, msg: str, exc: Optional[BaseException] = None) -> None:
        if level < self.loglevel and exc is None:
            return
        self.publish(LogEvent(level, source, msg, exc, time.time()))

    def publish_unhandled(self, msg: Any, recipient: ActorRef) -> None:
        self.publish_log(logging.DEBUG, recipient.path, f"unhandled message {msg!r}")


def python_logging_subscriber(ev: Any) -> None:
    if isinstance(ev, LogEvent):
        log_root.log(ev.level, "[%s] %s", ev.source, ev.message)


# ====================================================================== scheduler
class Scheduler:
    """Single timer thread (``system.scheduler.scheduleOnce``)."""

    def __init__(self):
        self._heap: List[Tuple[float, int, Callable[[], None]]] = []
        self._cv = threading.Condition()
        self._seq = itertools.count()
        self._stop = False
        self._t = threading.Thread(target=self._loop, name="actor-scheduler", daemon=True)
        self._t.start()

    def schedule_once(self, delay_s: float, fn: Callable[[], None]) -> Callable[[], None]:
        entry = [True]

        def run():
            if entry[0]:
                fn()

        with self._cv:
            item = (time.monotonic() + max(0.0, delay_s), next(self._seq), run)
            heapq.heappush(self._heap, item)
            if self._heap[0] is item:   # a new earliest deadline: the timer thread must re-arm (else no wake-up:
                self._cv.notify()       # an ask's 10 s timeout is almost never the earliest)

        def cancel():
            entry[0] = False

        return cancel

    def tell_once(self, delay_s: float, ref: ActorRef, msg: Any, sender: Optional[ActorRef] = None):
        return self.schedule_once(delay_s, lambda: ref.tell(msg, sender))

    def _loop(self) -> None:
        while True:
            with self._cv:
                while not self._stop and (not self._heap or self._heap[0][0] > time.monotonic()):
                    timeout = None if not self._heap else max(0.0, self._heap[0][0] - time.monotonic())
                    self._cv.wait(timeout)
                if self._stop:
                    return
                _, _, fn = heapq.heappop(self._heap)
            try:
                fn()
            except Exception:  # noqa: BLE001
                traceback.print_exc()

    def shutdown(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()


# ====================================================================== system
class ActorSystem:
    """Hosts actors on a thread-pool dispatcher (Akka's default dispatcher)."""

    def __init__(self, name: str = "sharetrade", threads: int = 8, loglevel: str = "INFO",
                 config=None, debug: Optional[bool] = None):
        self.name = name
        self.debug = bool(int(os.environ.get("SHARETRADE_ACTOR_DEBUG", "0"))) if debug is None else debug
        self.config = config
        lvl = getattr(logging, str(loglevel).upper(), logging.INFO)
        self.event_stream = EventStream(lvl)
        self.event_stream.subscribe(python_logging_subscriber)
        self._pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix=f"{name}-dispatcher")
        self.scheduler = Scheduler()
        self._top: Dict[str, ActorCell] = {}
        self._lock = threading.Lock()
        self._names = itertools.count()
        self._terminated = threading.Event()
        self.dead_letters = _FunctionRef(f"akka://{name}/deadLetters", self._dead_letter_tell)
        self._shutdown = False

    # ------------------------------------------------------------ dispatch
    def _execute(self, fn: Callable[[], None]) -> None:
        if self._shutdown:
            return
        try:
            self._pool.submit(fn)
        except RuntimeError:
            pass

    def dispatcher(self, fn: Callable[[], None]) -> None:
        self._execute(fn)

    def future(self, fn: Callable[[], Any]) -> Future:
        """``Future { ... }`` on a dispatcher thread."""
        f = Future(self._execute)

        def run():
            try:
                f.set_result(fn())
            except BaseException as e:  # noqa: BLE001
                f.set_exception(e)

        self._execute(run)
        return f

    def blocking_future(self, fn: Callable[[], Any], name: str = "blocking") -> Future:
        """A future run on its own thread (blocking work must not starve the dispatcher)."""
        f = Future(self._execute)

        def run():
            try:
                f.set_result(fn())
            except BaseException as e:  # noqa: BLE001
                f.set_exception(e)

        threading.Thread(target=run, name=f"{self.name}-{name}", daemon=True).start()
        return f

    # ------------------------------------------------------------ creation
    def actor_of(self, props: Props, name: Optional[str] = None) -> ActorRef:
        return self._spawn(props, name, None)

    def _spawn(self, props: Props, name: Optional[str], parent: Optional[ActorCell]) -> ActorRef:
        if name is None:
            name = f"$" + _base64_name(next(parent.child_counter if parent is not None else self._names))
        with self._lock:
            siblings = parent.children if parent is not None else self._top
            if name in siblings and not siblings[name].dead:
                raise ValueError(f"actor name [{name}] is not unique!")
            base = parent.ref.path if parent is not None else f"akka://{self.name}/user"
            cell = ActorCell(self, props, f"{base}/{name}", parent)
            siblings[name] = cell
        cell.create()
        return cell.ref

    # ------------------------------------------------------------ stopping
    def stop(self, ref: ActorRef) -> None:
        c = ref._cell
        if c is None or c.dead:
            return
        c.enqueue_system(_Stop)

    def _stop_cell(self, cell: ActorCell) -> None:
        if cell.dead or cell.stopping:
            return
        cell.stopping = True
        cell.suspended = True
        kids = list(cell.children.values())
        if not kids:
            self._finish_stop(cell)
            return
        for k in kids:
            self.stop(k.ref)

    def _finish_stop(self, cell: ActorCell) -> None:
        if cell.dead:
            return
        try:
            if cell.actor is not None:
                cell.actor.post_stop()
        except Exception:  # noqa: BLE001
            traceback.print_exc()
        with cell.lock:
            cell.dead = True
            pending = list(cell.mailbox)
            cell.mailbox.clear()
            watchers = list(cell.watchers)
        for msg, snd in pending:
            self._dead_letter(msg, snd, cell.ref)
        for w in watchers:
            w.tell(Terminated(cell.ref), cell.ref)
        if cell.parent is not None:
            cell.parent.enqueue_system(_ChildTerminated(cell.ref))
        else:
            with self._lock:
                for k, v in list(self._top.items()):
                    if v is cell:
                        del self._top[k]

    # ------------------------------------------------------------ ask / dead letters
    def _ask(self, target: ActorRef, msg: Any, timeout: float) -> Future:
        p = Future(self._execute)
        ref = _PromiseRef(self, f"akka://{self.name}/temp/${next(self._names)}", p)
        if timeout is not None and timeout > 0:
            cancel = self.scheduler.schedule_once(
                timeout, lambda: p.set_exception(AskTimeoutException(
                    f"Ask timed out on [{target.path}] after [{int(timeout * 1000)} ms]. "
                    f"Message of type [{type(msg).__name__}]")))
            p.on_complete(lambda _f: cancel(), inline=True)
        target.tell(msg, ref)
        return p

    def _dead_letter(self, msg: Any, sender: Optional[ActorRef], recipient: ActorRef) -> None:
        if msg is PoisonPill or isinstance(msg, Terminated):
            return
        self.event_stream.publish(DeadLetter(msg, sender, recipient))
        self.event_stream.publish_log(logging.DEBUG, recipient.path, f"dead letter {msg!r}")

    def _dead_letter_tell(self, msg: Any, sender: Optional[ActorRef]) -> None:
        self._dead_letter(msg, sender, self.dead_letters)

    # ------------------------------------------------------------ shutdown
    def terminate(self, timeout: float = 5.0) -> None:
        with self._lock:
            tops = list(self._top.values())
        for c in tops:
            self.stop(c.ref)
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            with self._lock:
                if not self._top:
                    break
            time.sleep(0.005)
        self._shutdown = True
        self.scheduler.shutdown()
        self._pool.shutdown(wait=False, cancel_futures=True)
        self._terminated.set()

    def when_terminated(self, timeout: Optional[float] = None) -> bool:
        return self._terminated.wait(timeout)

    def __enter__(self) -> "ActorSystem":
        return self

    def __exit__(self, *exc) -> None:
        self.terminate()


def _base64_name(n: int) -> str:
    alphabet = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789+~"
    s = ""
    while True:
        s += alphabet[n & 63]
        n >>= 6
        if n == 0:
            return s


# ====================================================================== patterns
def ask(ref: ActorRef, msg: Any, timeout: float = 10.0) -> Future:
    return ref.ask(msg, timeout)


def pipe_to(fut: Future, ref: ActorRef, sender: Optional[ActorRef] = None) -> Future:
    """``future pipeTo ref``: the value (or ``Status.Failure``) is sent as a message."""

    def cb(f: Future):
        v = f.value()
        if v[0] == "ok":
            ref.tell(v[1], sender)
        else:
            ref.tell(Status.Failure(v[1]), sender)

    fut.on_complete(cb)
    return fut
