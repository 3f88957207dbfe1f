"""``PolicyServingActor`` — the reference's ``SelectionAction`` API served from the GPU kernel.

Same message contract as ``QDecisionPolicyActor`` for decisions (``QDecisionPolicyActor.scala:
32,56-62``): ``SelectionAction(state [1,203], step)`` -> ``Buy`` | ``Sell`` | ``Hold``, and a state
that is not ``input_dim`` wide fails the actor with ``IllegalArgumentException`` (supervision
decides).  It does not learn: ``LoadPolicy(params)`` swaps in new weights (from a training engine
or a checkpoint) and replies ``PolicyLoaded``.  Selections already queued in the mailbox are
answered with one batched launch (a ``_Flush`` the actor sends itself lands behind them), and a
``LoadPolicy`` first answers the selections queued before it, so each decision sees the weights in
force when it arrived.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, List, Optional, Tuple

import torch

from ..actors.runtime import Actor, ActorRef, NotHandled, Props, singleton
from ..errors import IllegalArgumentException
from ..protocol import SelectionAction, action_of
from .server import PolicyServer

_Flush = singleton("PolicyServingActor._Flush")
PolicyLoaded = singleton("PolicyLoaded")


@dataclass(frozen=True, eq=False)
class LoadPolicy:
    params: Any   # fp32 flat params (engine layout)


class PolicyServingActor(Actor):
    def __init__(self, server: PolicyServer):
        self.server = server
        self.width = server.H + 2
        self._pending: List[Tuple[torch.Tensor, float, Optional[ActorRef]]] = []
        self._flush_scheduled = False

    @classmethod
    def props(cls, server: PolicyServer) -> Props:
        return Props(cls, server)

    def receive(self, msg: Any) -> Any:
        if isinstance(msg, SelectionAction):
            x = torch.as_tensor(msg.current_state, dtype=torch.float32)
            if x.numel() != self.width:
                who = self.sender.parent_name if self.sender is not None else "?"
                raise IllegalArgumentException(
                    f"SelectionAction received from {who}, but policy input size({self.width}) and "
                    f"state({x.numel()}) size do not match")
            self._pending.append((x.reshape(1, -1), float(msg.step), self.sender))
            if not self._flush_scheduled:
                self._flush_scheduled = True
                self.self_ref.tell(_Flush, self.self_ref)
            return None
        if msg is _Flush:
            self._flush_scheduled = False
            self._flush()
            return None
        if isinstance(msg, LoadPolicy):
            self._flush()
            self.server.load_params(torch.as_tensor(msg.params))
            if self.sender is not None:
                self.sender.tell(PolicyLoaded, self.self_ref)
            return None
        return NotHandled

    def _flush(self) -> None:
        if not self._pending:
            return
        pend, self._pending = self._pending, []
        acts = self.server.infer(torch.cat([p[0] for p in pend], 0), [p[1] for p in pend]).cpu().tolist()
        for (_, _, snd), a in zip(pend, acts):
            if snd is not None:
                snd.tell(action_of(int(a)), self.self_ref)

    def post_stop(self) -> None:
        self._flush()
