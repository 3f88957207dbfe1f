"""``TrainerChildActor`` — the Buy/Sell/Hold rollout worker FSM.

Reference (`TrainerChildActor.scala:26-163`)::

    Ready   + Train(data)      -> fold over N-201 steps (ask SelectionAction, ask UpdateQ) ; pipe TrainedData to self
    Ready   + TrainedData(p)   -> parent ! Trained ; goto Trained using TrainedData(p)
    Ready   + GetPortfolio     -> NotComputed
    Ready   + Initialise       -> log "already in ready state"
    Trained + Train            -> log "it's already trained"
    Trained + GetPortfolio     -> TrainedData(p)
    Trained + Initialise       -> parent ! Initialised ; goto Ready using NotComputed

One episode step ``i`` (`:87-102`): ``state = prices[i, i+H) ++ (b, s)``,
``action <- policy ? SelectionAction(state, i)``, trade at ``v = prices[i+H]``
(`makeDecisionAccordingToAction`, :118-123), reward = Δ portfolio,
``next = prices[i+1, i+H+1) ++ (b', s')``, ``policy ? UpdateQ(...)`` and wait
for ``Updated``.  Portfolio arithmetic is in float64 (Scala ``Double``), the
state tensors in float32, exactly as the reference builds them.

``env.compat_decisions=True`` reproduces quirk Q1 (decisions from the
constructor budget/shares); the default preset fixes it.  ``train`` is the
overridable seam the reference's router test replaces with a fake
(`TrainerRouterActorSpec.scala:144-153`).
"""
from __future__ import annotations

from typing import Any, Optional, Tuple

import numpy as np

from ..actors.fsm import FSM, Event
from ..actors.future import Future
from ..actors.runtime import ActorRef, NotHandled, Props, pipe_to
from ..config import Config, preset_config
from ..errors import IllegalArgumentException
from ..protocol import (GetPortfolio, Initialise, Initialised, NotComputed, Ready, SelectionAction, Train, Trained,
                        TrainedData, UpdateQ, Updated, Buy, Sell)


class TrainerChildActor(FSM):
    def __init__(self, policy_actor: ActorRef, my_budget: float, no_of_stocks: int, cfg: Optional[Config] = None):
        super().__init__()
        self.policy_actor = policy_actor
        self.my_budget = float(my_budget)
        self.no_of_stocks = int(no_of_stocks)
        self.cfg = cfg or preset_config("reference_compat")
        self.start_with(Ready, NotComputed)
        self.when(Ready, self._ready)
        self.when(Trained, self._trained)
        self.initialize()

    @classmethod
    def props(cls, policy_actor: ActorRef, budget: float, no_of_stocks: int, cfg: Optional[Config] = None) -> Props:
        return Props(cls, policy_actor, budget, no_of_stocks, cfg)

    def _tag(self) -> str:
        p = self.self_ref.parent_name
        return p[-1:] if p else "?"

    # ------------------------------------------------------------------ states
    def _ready(self, ev: Event):
        m, d = ev.msg, ev.data
        if isinstance(m, Train) and d is NotComputed:
            self.log.info(f"{self._tag()} training starts")
            fut = self.train(m.stock_data)
            pipe_to(fut.map(TrainedData), self.self_ref)
            return self.stay()
        if isinstance(m, TrainedData) and d is NotComputed:
            self.log.info(f"{self._tag()} training finished")
            parent = self.context.parent
            if parent is not None:
                parent.tell(Trained, self.self_ref)
            return self.goto(Trained).using(m)
        if m is GetPortfolio and d is NotComputed:
            self.sender.tell(NotComputed, self.self_ref)
            return self.stay()
        if m is Initialise and d is NotComputed:
            self.log.info(f"{self._tag()} is already in ready state")
            return self.stay()
        return NotHandled

    def _trained(self, ev: Event):
        m = ev.msg
        if isinstance(m, Train):
            self.log.info("it's already trained")
            return self.stay()
        if m is GetPortfolio and isinstance(ev.data, TrainedData):
            self.sender.tell(ev.data, self.self_ref)
            return self.stay()
        if m is Initialise:
            parent = self.context.parent
            if parent is not None:
                parent.tell(Initialised, self.self_ref)
            return self.goto(Ready).using(NotComputed)
        return NotHandled

    # ------------------------------------------------------------------ training
    def train(self, stock_data) -> Future:
        """Returns a future of the final portfolio.  Raises (synchronously, so the
        actor fails and supervision decides) when the series is too short."""
        prices = np.asarray(list(stock_data.share_prices.values()), dtype=np.float64)
        H = self.cfg.model.history
        if prices.size <= H:
            raise IllegalArgumentException("Stock price count should be more than Tensorflow input nodes")
        pf32 = prices.astype(np.float32)
        return self.context.system.blocking_future(lambda: self._episode(pf32), name="episode")

    def _episode(self, prices: np.ndarray) -> float:
        H = self.cfg.model.history
        n_steps = prices.size - H
        timeout = self.cfg.router.ask_timeout_s
        compat = self.cfg.env.compat_decisions
        every = self.cfg.env.progress_every
        b, s, v_prev = self.my_budget, self.no_of_stocks, 0.0
        v = 0.0
        for i in range(n_steps):
            if every and i % every == 0:
                self.log.info(f"{self._tag()} progress {100 * i // n_steps}%, index no: {i}")
            state = np.concatenate([prices[i:i + H], np.array([b, s], dtype=np.float32)]).astype(np.float32)
            cur = b + s * v_prev
            action = self.policy_actor.ask(SelectionAction(state[None, :], float(i)), timeout).result(timeout + 1)
            v = float(prices[i + H])
            nb, ns, _effective = self._decide(action, v, (self.my_budget, self.no_of_stocks) if compat else (b, s))
            taken = getattr(action, "index", 2)  # the Q(s, a) slot is the *selected* action
            reward = (nb + ns * v) - cur
            nxt = np.concatenate([prices[i + 1:i + H + 1], np.array([nb, ns], dtype=np.float32)]).astype(np.float32)
            act_idx = None if self.cfg.agent.target_slot == "compat" else taken
            reply = self.policy_actor.ask(UpdateQ(state[None, :], float(np.float32(reward)), nxt[None, :], act_idx),
                                          timeout).result(timeout + 1)
            if reply is not Updated:
                raise RuntimeError(f"unexpected UpdateQ reply {reply!r}")
            b, s, v_prev = nb, ns, v
        return b + s * v

    @staticmethod
    def _decide(action: Any, v: float, bs: Tuple[float, int]) -> Tuple[float, int, int]:
        """``makeDecisionAccordingToAction`` (`TrainerChildActor.scala:118-123`)."""
        b, s = bs
        if action is Buy and b >= v:
            return b - v, s + 1, 0
        if action is Sell and s > 0:
            return b + v, s - 1, 1
        return b, s, 2
