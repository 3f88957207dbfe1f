"""``TrainerRouterActor`` — broadcast fan-out, lifecycle, aggregation, fault tolerance.

Reference (`TrainerRouterActor.scala:40-151`):

* 10 children, each a ``BackoffSupervisor`` (3 s .. 1 min, jitter 0.2) around a
  ``TrainerChildActor`` with the directive map ArithmeticException→Resume,
  NullPointerException→Restart, IllegalArgumentException→Stop,
  Exception→Escalate; every wrapper is death-watched (`:46-64`);
* ``Router(BroadcastRoutingLogic)`` over the wrappers (`:66`);
* lifecycle with ``Stash`` (`:68-130`)::

    awaitingTrainingData --SendTrainingData--> trainingDataPresent --Trained--> trained(n) --10th Trained--> completed

* ``GetAvg``/``GetStd``: ask every *trained* child ``GetPortfolio`` and reduce
  to mean / population std (`:89-94,137-139,148-151`);
* ``Terminated(ref)``: replace the routee (`:101-102,116-120,141-146`).

Default (intended) behaviour fixes the reference's quirks Q9 (reply
``Result(x)`` instead of a bare ``Double``) and Q14 (a replaced worker is
re-sent ``Train`` once training has started, and a death in ``trained`` always
installs the replacement); ``RouterConfig.reply_result`` /
``redispatch_on_restart`` switch back to the reference's behaviour.
"""
from __future__ import annotations

import math
from typing import Any, List, Optional, Sequence

from ..actors.backoff import Backoff, BackoffSupervisor
from ..actors.future import Future, sequence
from ..actors.routing import BroadcastRoutingLogic, GetRoutees, Router
from ..actors.runtime import (Actor, ActorRef, Escalate, NotHandled, OneForOneStrategy, Props, Restart, Resume,
                              Stash, Stop, Terminated, pipe_to)
from ..config import Config, preset_config
from ..errors import ArithmeticException, IllegalArgumentException, NullPointerException
from ..protocol import (Completed, Died, GetAvg, GetPortfolio, GetStd, IsEverythingDone, NoTrainingDataReceived,
                        NotComputed, Result, SendTrainingData, StartTraining, Train, Trained, TrainedData,
                        TrainingNotCompleted)
from .child import TrainerChildActor

NO_OF_CHILDREN = 10  # TrainerRouterActor.scala:36

CHILD_DECIDER = [
    (ArithmeticException, Resume),
    (NullPointerException, Restart),
    (IllegalArgumentException, Stop),
    (Exception, Escalate),
]


def mean(xs: Sequence[float]) -> float:
    return float(sum(xs)) / len(xs) if xs else float("nan")


def std_dev(xs: Sequence[float]) -> float:
    """Population standard deviation (`TrainerRouterActor.scala:148-151`), two-pass."""
    if not xs:
        return float("nan")
    m = mean(xs)
    return math.sqrt(sum((x - m) ** 2 for x in xs) / len(xs))


class TrainerRouterActor(Actor, Stash):
    def __init__(self, policy_actor: ActorRef, budget: float, no_of_stocks: int, cfg: Optional[Config] = None,
                 child_trainer_props: Optional[Props] = None, n_children: Optional[int] = None):
        self.policy_actor = policy_actor
        self.budget = float(budget)
        self.no_of_stocks = int(no_of_stocks)
        self.cfg = cfg or preset_config("reference_compat")
        rc = self.cfg.router
        self.n_children = int(n_children if n_children is not None else rc.n_workers)
        # test seam: `lazy val childTrainerProp` (TrainerRouterActor.scala:44)
        self.child_trainer_props = child_trainer_props or self.make_child_trainer_props()
        self.child_props = BackoffSupervisor.props(
            Backoff.on_failure(self.child_trainer_props, "child-trainer", rc.backoff_min_s, rc.backoff_max_s,
                               rc.backoff_jitter).with_supervisor_strategy(OneForOneStrategy(CHILD_DECIDER)))
        self.training_started = False

    def make_child_trainer_props(self) -> Props:
        return TrainerChildActor.props(self.policy_actor, self.budget, self.no_of_stocks, self.cfg)

    def pre_start(self) -> None:
        children = []
        for i in range(self.n_children):
            c = self.context.actor_of(self.child_props, f"child_trainer_supervisor_wrapped{i}")
            self.context.watch(c)
            children.append(c)
        self.context.become(self._awaiting(Router(BroadcastRoutingLogic(), children)))

    # ------------------------------------------------------------------ helpers
    def _reply_value(self, x: float):
        return Result(x) if self.cfg.router.reply_result else x

    def _get_routees(self, msg: Any, router: Router) -> bool:
        if msg is GetRoutees:
            self.sender.tell(router.get_routees(), self.self_ref)
            return True
        return False

    def _compute_portfolios(self, actors: Sequence[ActorRef]) -> Future:
        t = self.cfg.router.ask_timeout_s
        futs = [a.ask(GetPortfolio, t) for a in actors]
        return sequence(futs, self.context.system.dispatcher).map(
            lambda rs: [r.portfolio for r in rs if isinstance(r, TrainedData)])

    def _create_new_child_when_terminated(self, ref: ActorRef, router: Router, data=None) -> Router:
        cleaned = router.remove_routee(ref)
        child = self.context.actor_of(self.child_props)
        self.context.watch(child)
        if data is not None and self.training_started and self.cfg.router.redispatch_on_restart:
            child.tell(Train(data), self.self_ref)
        return cleaned.add_routee(child)

    # ------------------------------------------------------------------ states
    def _awaiting(self, router: Router):
        def behave(msg: Any):
            if self._get_routees(msg, router):
                return None
            if isinstance(msg, SendTrainingData):
                self.log.info("training data received")
                self.unstash_all()
                self.context.become(self._training_data_present(msg.stock_data, router))
                return None
            if msg is GetStd or msg is GetAvg or msg is IsEverythingDone:
                self.sender.tell(NoTrainingDataReceived, self.self_ref)
                return None
            if msg is StartTraining:
                self.stash()
                return None
            if isinstance(msg, Terminated):
                self.context.become(self._awaiting(self._create_new_child_when_terminated(msg.actor, router)))
                return None
            self.log.info(f"unknown : {msg!r} message received")
            self.stash()
            return None
        return behave

    def _common(self, msg: Any, data, actors: Optional[List[ActorRef]], router: Router) -> bool:
        if self._get_routees(msg, router):
            return True
        if msg is StartTraining:
            self.log.info("training start")
            self.training_started = True
            router.route(Train(data), self.sender)
            return True
        if msg is GetStd or msg is GetAvg:
            fn = std_dev if msg is GetStd else mean
            if actors is None:
                fut = Future.successful(NotComputed)
            else:
                fut = self._compute_portfolios(actors).map(lambda ps: self._reply_value(fn(ps)))
            pipe_to(fut, self.sender)
            return True
        return False

    def _training_data_present(self, data, router: Router):
        def behave(msg: Any):
            if self._common(msg, data, None, router):
                return None
            if msg is IsEverythingDone:
                self.sender.tell(NotComputed, self.self_ref)
                return None
            if isinstance(msg, Terminated):
                self.context.become(self._training_data_present(
                    data, self._create_new_child_when_terminated(msg.actor, router, data)))
                return None
            if msg is Trained:
                self.unstash_all()
                snd = self.sender
                nxt = [snd]
                r2 = router.remove_routee(snd)
                if len(nxt) >= self.n_children:
                    self.context.become(self._completed(data, nxt, r2))
                else:
                    self.context.become(self._trained(data, nxt, r2))
                return None
            self.stash()
            return None
        return behave

    def _trained(self, data, actors: List[ActorRef], router: Router):
        def behave(msg: Any):
            if self._common(msg, data, actors, router):
                return None
            if msg is Trained:
                trained = actors + [self.sender]
                cleaned = router.remove_routee(self.sender)
                if len(trained) >= self.n_children:
                    self.context.become(self._completed(data, trained, cleaned))
                else:
                    self.context.become(self._trained(data, trained, cleaned))
                return None
            if isinstance(msg, Terminated):
                if self.cfg.router.redispatch_on_restart:
                    new_router = self._create_new_child_when_terminated(msg.actor, router, data)
                    self.context.become(self._trained(data, [a for a in actors if a != msg.actor], new_router))
                else:
                    # reference: self ! Died(ref, newRouter); self ! StartTraining (:116-118)
                    new_router = self._create_new_child_when_terminated(msg.actor, router)
                    self.self_ref.tell(Died(msg.actor, new_router), self.self_ref)
                    self.self_ref.tell(StartTraining, self.self_ref)
                return None
            if isinstance(msg, Died):
                if msg.ref in actors:
                    self.context.become(self._trained(data, [a for a in actors if a != msg.ref], msg.router))
                return None
            if msg is IsEverythingDone:
                self.sender.tell(TrainingNotCompleted, self.self_ref)
                return None
            return NotHandled
        return behave

    def _completed(self, data, actors: List[ActorRef], router: Router):
        def behave(msg: Any):
            if self._common(msg, data, actors, router):
                return None
            if msg is IsEverythingDone:
                self.log.info("Completed")
                self.sender.tell(Completed, self.self_ref)
                return None
            if isinstance(msg, Terminated):
                if msg.actor in actors and self.cfg.router.redispatch_on_restart:
                    new_router = self._create_new_child_when_terminated(msg.actor, router, data)
                    self.context.become(self._trained(data, [a for a in actors if a != msg.actor], new_router))
                return None
            return NotHandled
        return behave

    def receive(self, msg: Any) -> Any:  # replaced in pre_start
        return NotHandled

    @classmethod
    def props(cls, policy_actor: ActorRef, budget: float, no_of_stocks: int, cfg: Optional[Config] = None,
              **kw) -> Props:
        return Props(cls, policy_actor, budget, no_of_stocks, cfg, **kw)
