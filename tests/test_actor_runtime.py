"""Actor-runtime semantics the reference relies on (Akka): tell/ask, become,
stash, death watch, supervision directives, backoff supervision, FSM, routers."""
import threading
import time

import pytest

from sharetrade.actors import backoff as bo
from sharetrade.actors.fsm import FSM
from sharetrade.actors.future import AskTimeoutException, Future, sequence
from sharetrade.actors.routing import BroadcastRoutingLogic, RoundRobinRoutingLogic, Router
from sharetrade.actors.runtime import (Actor, ActorSystem, Escalate, NotHandled, OneForOneStrategy, PoisonPill, Props,
                                       Restart, Resume, Stash, Status, Stop, Terminated, pipe_to)
from sharetrade.actors.testkit import EventFilter, TestKit, TestProbe, await_assert


@pytest.fixture
def system():
    s = ActorSystem("test", loglevel="DEBUG")
    yield s
    s.terminate()


class Echo(Actor):
    def receive(self, msg):
        self.sender.tell(msg, self.self_ref)


class Counter(Actor):
    def __init__(self):
        self.n = 0

    def receive(self, msg):
        if msg == "inc":
            self.n += 1
        elif msg == "get":
            self.sender.tell(self.n, self.self_ref)
        elif msg == "boom":
            raise RuntimeError("boom")
        elif msg == "arith":
            raise ArithmeticError("arith")
        elif msg == "value":
            raise ValueError("value")
        else:
            return NotHandled


def test_tell_ask_and_order(system):
    kit = TestKit(system)
    e = system.actor_of(Props(Echo), "echo")
    for i in range(50):
        kit.tell(e, i)
    assert kit.receive_n(50) == list(range(50))
    assert e.ask("hi", 1.0).result(2) == "hi"


def test_ask_timeout(system):
    class Silent(Actor):
        def receive(self, msg):
            return None

    s = system.actor_of(Props(Silent))
    with pytest.raises(AskTimeoutException):
        s.ask("x", 0.1).result(2)


def test_status_failure_fails_ask(system):
    class Failer(Actor):
        def receive(self, msg):
            self.sender.tell(Status.Failure(KeyError("k")), self.self_ref)

    f = system.actor_of(Props(Failer)).ask("x", 1.0)
    with pytest.raises(KeyError):
        f.result(2)


def test_become_and_stash(system):
    class Gate(Actor, Stash):
        def receive(self, msg):
            if msg == "open":
                self.unstash_all()
                self.context.become(self.opened)
            else:
                self.stash()

        def opened(self, msg):
            self.sender.tell(("got", msg), self.self_ref)

    kit = TestKit(system)
    g = system.actor_of(Props(Gate))
    kit.tell(g, 1)
    kit.tell(g, 2)
    kit.expect_no_message(0.1)
    kit.tell(g, "open")
    assert kit.receive_n(2) == [("got", 1), ("got", 2)]


def test_default_supervision_restarts(system):
    c = system.actor_of(Props(Counter))
    c.tell("inc")
    c.tell("inc")
    assert c.ask("get").result(2) == 2
    c.tell("boom")
    await_assert(lambda: _eq(c.ask("get").result(2), 0), 2.0)   # fresh instance after restart


def _eq(a, b):
    assert a == b


def test_directives_resume_restart_stop_escalate(system):
    events = []

    class Parent(Actor):
        supervisor_strategy = OneForOneStrategy([(ArithmeticError, Resume), (ValueError, Stop),
                                                 (RuntimeError, Restart), (Exception, Escalate)])

        def pre_start(self):
            self.child = self.context.watch(self.context.actor_of(Props(Counter), "c"))

        def receive(self, msg):
            if isinstance(msg, Terminated):
                events.append("terminated")
            elif msg == "child?":
                self.sender.tell(self.child, self.self_ref)

    p = system.actor_of(Props(Parent), "parent")
    child = p.ask("child?").result(2)
    child.tell("inc")
    child.tell("arith")                          # Resume: state kept
    await_assert(lambda: _eq(child.ask("get").result(2), 1))
    child.tell("boom")                           # Restart: state reset
    await_assert(lambda: _eq(child.ask("get").result(2), 0))
    child.tell("value")                          # Stop
    await_assert(lambda: _eq(events, ["terminated"]))
    assert child.is_terminated()


def test_death_watch_and_poison_pill(system):
    probe = TestProbe(system)
    e = system.actor_of(Props(Echo))
    probe.watch(e)
    e.tell(PoisonPill)
    probe.expect_terminated(e)


def test_dead_letters_after_stop(system):
    got = []
    system.event_stream.subscribe(lambda ev: got.append(ev) if type(ev).__name__ == "DeadLetter" else None)
    e = system.actor_of(Props(Echo))
    system.stop(e)
    await_assert(lambda: _eq(e.is_terminated(), True))
    e.tell("late")
    await_assert(lambda: _eq(len(got), 1))


def test_backoff_supervisor_restarts_with_delay(system):
    class Flaky(Actor):
        created = []

        def pre_start(self):
            Flaky.created.append(time.monotonic())

        def receive(self, msg):
            if msg == "npe":
                raise RuntimeError("npe")
            self.sender.tell(("child", msg), self.self_ref)

    opts = bo.Backoff.on_failure(Props(Flaky), "child", 0.2, 1.0, 0.0).with_supervisor_strategy(
        OneForOneStrategy([(RuntimeError, Restart)]))
    kit = TestKit(system)
    sup = system.actor_of(bo.BackoffSupervisor.props(opts), "sup")
    kit.tell(sup, "hello")                       # forwarded to the child, reply goes to us
    assert kit.expect_msg(("child", "hello"))
    kit.tell(sup, "npe")
    await_assert(lambda: _eq(len(Flaky.created), 2), 3.0, 0.02)
    assert Flaky.created[1] - Flaky.created[0] >= 0.19   # min backoff honoured
    kit.tell(sup, bo.GetRestartCount)
    assert kit.expect_msg_type(bo.RestartCount).count == 1


def test_backoff_delay_formula():
    assert bo.calculate_delay(0, 3, 60, 0.0) == 3
    assert bo.calculate_delay(3, 3, 60, 0.0) == 24
    assert bo.calculate_delay(10, 3, 60, 0.0) == 60
    for n in range(6):
        d = bo.calculate_delay(n, 3, 60, 0.2)
        base = min(60, 3 * 2 ** n)
        assert base <= d <= base * 1.2


def test_backoff_child_messages_go_to_parent_with_wrapper_as_sender(system):
    class Child(Actor):
        def receive(self, msg):
            self.context.parent.tell(("up", msg), self.self_ref)

    probe = TestProbe(system)
    opts = bo.Backoff.on_failure(Props(Child), "child-trainer", 3, 60, 0.2)
    from sharetrade.actors.testkit import TestActorRef

    sup = TestActorRef(system, bo.BackoffSupervisor.props(opts), probe.ref, "wrapped0")
    sup.tell("x")
    assert probe.expect_msg(("up", "x"))
    assert probe.last_sender == sup


def test_backoff_child_stop_stops_wrapper(system):
    probe = TestProbe(system)
    opts = bo.Backoff.on_failure(Props(Counter), "c", 0.1, 1, 0.2).with_supervisor_strategy(
        OneForOneStrategy([(ValueError, Stop)]))
    sup = system.actor_of(bo.BackoffSupervisor.props(opts))
    probe.watch(sup)
    sup.tell("value")
    probe.expect_terminated(sup)


def test_fsm_transitions(system):
    class Light(FSM):
        def __init__(self):
            super().__init__()
            self.start_with("off", 0)
            self.when("off", self.off)
            self.when("on", self.on)
            self.initialize()

        def off(self, ev):
            if ev.msg == "toggle":
                return self.goto("on").using(ev.data + 1)
            if ev.msg == "state":
                return self.stay().replying(("off", ev.data))
            return NotHandled

        def on(self, ev):
            if ev.msg == "toggle":
                return self.goto("off")
            if ev.msg == "state":
                return self.stay().replying(("on", ev.data))
            return NotHandled

    kit = TestKit(system)
    l = system.actor_of(Props(Light))
    kit.tell(l, "state")
    kit.expect_msg(("off", 0))
    kit.tell(l, "toggle")
    kit.tell(l, "state")
    kit.expect_msg(("on", 1))
    kit.tell(l, "toggle")
    kit.tell(l, "state")
    kit.expect_msg(("off", 1))


def test_router_logics(system):
    kit = TestKit(system)
    probes = [TestProbe(system) for _ in range(3)]
    r = Router(BroadcastRoutingLogic(), [p.ref for p in probes])
    r.route("all", kit.ref)
    for p in probes:
        p.expect_msg("all")
        assert p.last_sender == kit.ref
    rr = Router(RoundRobinRoutingLogic(), [p.ref for p in probes])
    for i in range(6):
        rr.route(i)
    assert [probes[0].receive_one(), probes[0].receive_one()] == [0, 3]
    r2 = r.remove_routee(probes[1].ref).add_routee(probes[1].ref)
    assert [x.ref for x in r2.routees] == [probes[0].ref, probes[2].ref, probes[1].ref]
    assert len(r.routees) == 3   # immutable


def test_futures_compose(system):
    f = system.future(lambda: 2).map(lambda x: x * 3).flat_map(lambda x: Future.successful(x + 1))
    assert f.result(2) == 7
    s = sequence([system.future(lambda i=i: i) for i in range(5)])
    assert s.result(2) == [0, 1, 2, 3, 4]
    bad = system.future(lambda: 1 / 0).recover(lambda e: "recovered")
    assert bad.result(2) == "recovered"


def test_pipe_to(system):
    kit = TestKit(system)
    pipe_to(system.future(lambda: 42), kit.ref)
    kit.expect_msg(42)
    pipe_to(system.future(lambda: 1 / 0), kit.ref)
    m = kit.expect_msg_type(Status.Failure)
    assert isinstance(m.cause, ZeroDivisionError)


def test_event_filter_counts_exceptions(system):
    c = system.actor_of(Props(Counter))
    with EventFilter(system, ValueError, occurrences=1).intercept():
        c.tell("value")


def test_one_message_at_a_time(system):
    class Racy(Actor):
        def __init__(self):
            self.inside = 0
            self.max_inside = 0

        def receive(self, msg):
            if msg == "get":
                self.sender.tell(self.max_inside, self.self_ref)
                return
            self.inside += 1
            self.max_inside = max(self.max_inside, self.inside)
            time.sleep(0.0005)
            self.inside -= 1

    r = system.actor_of(Props(Racy))
    ts = [threading.Thread(target=lambda: [r.tell(i) for i in range(100)]) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert r.ask("get", 10).result(15) == 1
