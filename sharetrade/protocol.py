"""The public message API — source-compatible with the reference's sealed ADTs.

=========================  ==================================================  ==========================================
message                    meaning                                             reference
=========================  ==================================================  ==========================================
``Buy`` ``Sell`` ``Hold``  actions, index order 0, 1, 2                        QDecisionPolicyActor.scala:17,26-29
``SelectionAction``        state [1,203] + step -> an ``Action``              QDecisionPolicyActor.scala:32
``UpdateQ``                (state, reward, next_state[, action]) -> Updated    QDecisionPolicyActor.scala:33-34
``Train``                  start an episode over the stock data                TrainerChildActor.scala:19
``GetPortfolio``           -> ``NotComputed`` / ``TrainedData(p)``             TrainerChildActor.scala:15,42-44,54-56
``Initialise``             reset a trained worker -> ``Initialised``           TrainerChildActor.scala:16-17,45-47,57-59
``SendTrainingData``       hand the router its price data                      TrainerRouterActor.scala:16
``StartTraining``          broadcast ``Train`` to the workers                  TrainerRouterActor.scala:17
``GetAvg`` ``GetStd``      mean / population std of final portfolios           TrainerRouterActor.scala:18-19,89-94
``IsEverythingDone``       router lifecycle query                              TrainerRouterActor.scala:20
``RequestStockPrice``      (name, from, to) -> ``StockDataResponse``           SharePriceGetter.scala:14-15
``Event``                  the persisted price-query event                     SharePriceGetter.scala:17
=========================  ==================================================  ==========================================

``UpdateQ`` carries an optional ``action`` (the taken action): the reference's
3-field form cannot say which action was taken (quirk Q2), the intended
semantics need it.  ``Result(x)`` is what ``GetAvg``/``GetStd`` reply once
computed (quirk Q9 fixed; ``RouterConfig.reply_result=False`` replies the
reference's bare float).
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, Optional, Tuple

from .actors.runtime import ActorRef, _Singleton
from .persist import serialization


class _Msg(_Singleton):
    pass


def _obj(name: str, *bases):
    cls = type(name, bases or (_Msg,), {"_name": name})
    return cls()


# ---------------------------------------------------------------- actions
class Action(_Msg):
    index = -1


def _action(name: str, idx: int) -> Action:
    cls = type(name, (Action,), {"_name": name, "index": idx})
    return cls()


Buy = _action("Buy", 0)
Sell = _action("Sell", 1)
Hold = _action("Hold", 2)
ACTIONS: Tuple[Action, Action, Action] = (Buy, Sell, Hold)


def action_of(i: int) -> Action:
    return ACTIONS[int(i)]


# ---------------------------------------------------------------- decision policy
class DecisionPolicy:
    pass


@dataclass(frozen=True, eq=False)
class SelectionAction(DecisionPolicy):
    current_state: Any   # [1, 203] tensor-like (torch / numpy / list)
    step: float


@dataclass(frozen=True, eq=False)
class UpdateQ(DecisionPolicy):
    state: Any
    reward: float
    next_state: Any
    action: Optional[int] = None   # intended semantics (quirk Q2); None in the reference's 3-field form


class _Updated(_Msg, DecisionPolicy):
    _name = "Updated"


Updated = _Updated()


# ---------------------------------------------------------------- trainer states / data
class TrainerState:
    pass


class TrainerData:
    pass


def _state(name: str, *extra):
    cls = type(name, (_Msg, TrainerState) + extra, {"_name": name})
    return cls()


Ready = _state("Ready")
NoTrainingDataReceived = _state("NoTrainingDataReceived")
Trained = _state("Trained")
TrainingNotCompleted = _state("TrainingNotCompleted")
Completed = _state("Completed")
NotComputed = _state("NotComputed", TrainerData)


@dataclass(frozen=True)
class Result(TrainerData, TrainerState):
    double: float


@dataclass(frozen=True)
class TrainedData(TrainerData):
    portfolio: float


# ---------------------------------------------------------------- trainer child
GetPortfolio = _obj("GetPortfolio")
Initialise = _obj("Initialise")
Initialised = _obj("Initialised")


@dataclass(frozen=True, eq=False)
class Train:
    stock_data: "StockDataResponse"


# ---------------------------------------------------------------- router
class Trainer:
    pass


@dataclass(frozen=True, eq=False)
class SendTrainingData(Trainer):
    stock_data: "StockDataResponse"


StartTraining = _obj("StartTraining")
GetAvg = _obj("GetAvg")
GetStd = _obj("GetStd")
IsEverythingDone = _obj("IsEverythingDone")


@dataclass(frozen=True, eq=False)
class Died:
    ref: ActorRef
    router: Any


# ---------------------------------------------------------------- price getter
class TreeMap(dict):
    """Date-sorted immutable-ish mapping (``scala.collection.immutable.TreeMap``)."""

    def __init__(self, items: Iterable = ()):
        if isinstance(items, dict):
            items = items.items()
        super().__init__(sorted(items, key=lambda kv: kv[0]))

    def dates(self):
        return list(self.keys())

    def prices(self):
        return list(self.values())

    def __repr__(self) -> str:
        return f"TreeMap({dict.__repr__(self)})"


@dataclass(frozen=True)
class RequestStockPrice:
    stock_name: str
    from_: _dt.date
    to: _dt.date


@dataclass(frozen=True, eq=True)
class StockDataResponse:
    stock_name: str
    share_prices: TreeMap = field(default_factory=TreeMap)

    def __hash__(self) -> int:
        return hash((self.stock_name, len(self.share_prices)))

    @property
    def size(self) -> int:
        return len(self.share_prices)


@dataclass(frozen=True, eq=True)
class Event:
    stock_name: str
    share_prices: Dict[_dt.date, float]

    def __hash__(self) -> int:
        return hash((self.stock_name, len(self.share_prices)))


serialization.register(Event, 64, lambda e: (e.stock_name, dict(e.share_prices)),
                       lambda t: Event(t[0], dict(t[1])))
