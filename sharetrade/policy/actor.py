"""``QDecisionPolicyActor`` — the shared learner behind the message API.

Reference (`QDecisionPolicyActor.scala:36-94`): one actor owns the TF session;
``SelectionAction(state, step)`` replies an ``Action``; ``UpdateQ(state,
reward, nextState)`` trains once and replies ``Updated``; both throw
``IllegalArgumentException`` when a state is not 203 wide (-> the actor fails,
supervision decides); every 500 updates it calls an empty ``saveSnapshot``.

MI355X-first differences (semantics preserved):

* **Mailbox micro-batching.**  ``SelectionAction``s that are already queued
  are answered with ONE batched forward: a selection is held until a ``_Flush``
  the actor sends itself, which lands behind everything queued so far (with an
  empty mailbox it is answered at once: nothing could join the batch); any
  ``UpdateQ`` first flushes the pending selections, so every selection still
  sees exactly the weights it would have seen one-message-at-a-time.
* **Real snapshots.**  Every ``snapshot_interval`` updates the learner state is
  written with the deterministic C++ checkpoint writer and restored on start
  (quirk Q13 fixed) when ``checkpoint_dir`` is given.
"""
from __future__ import annotations

import os
from typing import Any, List, Optional, Tuple

import torch

from ..actors.runtime import Actor, ActorRef, NotHandled, Props, singleton
from ..config import Config, preset_config
from ..errors import IllegalArgumentException
from ..persist.checkpoint import CheckpointManager, load as load_ckpt
from ..protocol import SelectionAction, UpdateQ, Updated, action_of
from .learner import QLearner, as_state

_Flush = singleton("QDecisionPolicyActor._Flush")


class QDecisionPolicyActor(Actor):
    def __init__(self, cfg: Optional[Config] = None, device: Optional[torch.device] = None,
                 learner: Optional[QLearner] = None, checkpoint_dir: Optional[str] = None,
                 batch_selections: bool = True):
        self.cfg = cfg or preset_config("reference_compat")
        self.learner = learner or QLearner(self.cfg, device=device)
        self.input_dim = self.cfg.model.input_dim
        self.batch_selections = batch_selections
        self._pending: List[Tuple[torch.Tensor, float, Optional[ActorRef]]] = []
        self._flush_scheduled = False
        self.ckpt = CheckpointManager(checkpoint_dir, interval=self.cfg.agent.snapshot_interval) \
            if checkpoint_dir else None
        self.snapshots_saved = 0

    @classmethod
    def props(cls, cfg: Optional[Config] = None, **kw) -> Props:
        return Props(cls, cfg, **kw)

    # ------------------------------------------------------------------ lifecycle
    def pre_start(self) -> None:
        if self.ckpt is not None:
            p = self.ckpt.latest()
            if p is not None:
                state, meta = load_ckpt(p)
                self.learner.load_state_dict(state)
                self.log.info(f"policy restored from {os.path.basename(p)} (iteration {self.learner.iteration})")

    # ------------------------------------------------------------------ behaviour
    def receive(self, msg: Any) -> Any:
        if isinstance(msg, SelectionAction):
            st = self._check(msg.current_state, "state")
            if not self.batch_selections:
                a = self.learner.select(st, float(msg.step))[0]
                self.sender.tell(action_of(a), self.self_ref)
                return None
            self._pending.append((st, float(msg.step), self.sender))
            if not self._flush_scheduled:
                if self.context.mailbox_size() == 0:
                    self._flush()        # nothing queued to batch with: answer now (no _Flush round trip)
                else:
                    self._flush_scheduled = True
                    self.self_ref.tell(_Flush, self.self_ref)
            return None
        if msg is _Flush:
            self._flush_scheduled = False
            self._flush()
            return None
        if isinstance(msg, UpdateQ):
            s = self._check(msg.state, "state")
            ns = self._check(msg.next_state, "nextState")
            self._flush()
            it = self.learner.iteration
            self.learner.update(s, float(msg.reward), ns, msg.action, return_loss=False)
            # QDecisionPolicyActor.scala:74 — checked on the pre-increment counter
            if it % self.cfg.agent.snapshot_interval == 0 and it != 0:
                self.save_snapshot()
            if self.sender is not None:
                self.sender.tell(Updated, self.self_ref)
            return None
        return NotHandled

    def _check(self, state: Any, what: str) -> torch.Tensor:
        t = as_state(state, self.input_dim, what) if _numel(state) == self.input_dim else None
        if t is None:
            who = self.sender.parent_name if self.sender is not None else "?"
            raise IllegalArgumentException(
                f"{'SelectionAction' if what == 'state' else 'update q'} received from {who}, but tensorflow "
                f"input size({self.input_dim}) and {what}({_numel(state)}) size do not match")
        return t

    def _flush(self) -> None:
        if not self._pending:
            return
        pend, self._pending = self._pending, []
        x = torch.cat([p[0] for p in pend], 0)
        acts = self.learner.select(x, [p[1] for p in pend])
        for (_, _, snd), a in zip(pend, acts):
            if snd is not None:
                snd.tell(action_of(int(a)), self.self_ref)

    def save_snapshot(self) -> None:
        if self.ckpt is None:
            return
        self.ckpt.save(self.learner.iteration, self.learner.state_dict(),
                       {"kind": "QDecisionPolicyActor", "preset_hidden": list(self.cfg.model.hidden)})
        self.snapshots_saved += 1

    def post_stop(self) -> None:
        self._flush()


def _numel(x: Any) -> int:
    if isinstance(x, torch.Tensor):
        return x.numel()
    try:
        import numpy as np

        return int(np.asarray(x).size)
    except Exception:  # noqa: BLE001
        return -1
