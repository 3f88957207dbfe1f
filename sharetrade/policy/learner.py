"""QLearner — the Q-network learner behind ``QDecisionPolicyActor``.

Reference (`QDecisionPolicyActor.scala:38-77`):

* select: ``if U[0,1) < min(eps, step/1000): argmax q(state) else uniform{0,1,2}``;
* update: ``qS = q(state)``, ``qN = q(next)``, ``a* = argmax qN``,
  ``y = qS; y[a*] = r + gamma * qN[a*]``, one AdaGrad step on ``sum((y - q(state))^2)``.

The learner keeps the flat-parameter layout of :mod:`sharetrade.models.qnet`
(so the same checkpoint / all-reduce / kernel paths apply) and runs on one of
two backends:

* ``native`` — the fp32 HIP kernels of `csrc/mlp_f32.hip` (exact fp32 MFMA
  ``v_mfma_f32_16x16x4_f32``; forward+argmax, fused TD update + optimizer) on
  a GPU; required whenever the learner lives on a GPU;
* ``torch`` — the plain-PyTorch fp32 oracle on the CPU.

Batches are supported throughout (``[B, 203]``): the policy actor micro-batches
``SelectionAction`` messages that queue up in its mailbox.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Union

import numpy as np
import torch

from ..config import Config
from ..errors import IllegalArgumentException
from ..models import qnet as qn
from ..utils import rng

ArrayLike = Union[torch.Tensor, np.ndarray, Sequence[float]]


def as_state(x: ArrayLike, input_dim: int, what: str = "state") -> torch.Tensor:
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x, dtype=np.float32))
    t = t.detach().to(torch.float32)
    if t.numel() % input_dim != 0 or t.numel() == 0:
        raise IllegalArgumentException(
            f"tensorflow input size({input_dim}) and {what}({t.numel()}) size do not match")
    return t.reshape(-1, input_dim)


class QLearner:
    def __init__(self, cfg: Config, device: Optional[torch.device] = None, backend: str = "auto",
                 seed: Optional[int] = None, params: Optional[torch.Tensor] = None):
        self.cfg = cfg
        m, a = cfg.model, cfg.agent
        self.layout = qn.QNetLayout.from_config(m)
        self.input_dim = m.input_dim
        dev = device if device is not None else torch.device("cpu")
        self.device = dev
        if backend == "auto":
            backend = "native" if dev.type == "cuda" else "torch"
        if backend == "native" and dev.type != "cuda":
            raise ValueError("native learner backend needs a GPU device")
        self.backend = backend
        self.seed = a.seed if seed is None else seed
        p = params.clone().float() if params is not None else qn.init_params(self.layout, m, seed=self.seed, device=dev)
        self.params = p.to(dev)
        self.mask = self.layout.trainable_mask(m.train_bias).to(dev)
        self.opt = qn.OptimState(a.optimizer, self.layout.numel, a.adagrad_init_acc, device=dev)
        self.rng = rng.PhiloxStream(self.seed, stream=3)
        self.iteration = 0
        self._last_loss = 0.0
        self._loss_dev: Optional[torch.Tensor] = None
        self._k = None
        if backend == "native":
            from ..ops import mlp_f32

            self._k = mlp_f32.F32Learner(self)

    # ------------------------------------------------------------------ inference
    def q_values(self, states: ArrayLike) -> torch.Tensor:
        x = as_state(states, self.input_dim)
        if self._k is not None:   # host rows are staged by the kernel wrapper
            return self._k.forward(x)[:, : self.layout.n_actions]
        x = x.to(self.device)
        q, _, _ = qn.forward(self.params, self.layout, x, self.cfg.model.output_relu)
        return q[:, : self.layout.n_actions]

    def select(self, states: ArrayLike, steps) -> np.ndarray:
        """Epsilon-greedy actions for a batch (``QDecisionPolicyActor.scala:58-62``).

        Draw order per row: one uniform for the explore/exploit test, then (only
        when exploring) one for the random action — a seeded Philox stream
        instead of the reference's unseeded ``scala.util.Random`` (quirk Q8)."""
        x = as_state(states, self.input_dim)
        B = x.shape[0]
        steps = np.broadcast_to(np.asarray(steps, dtype=np.float32), (B,))
        a = self.cfg.agent
        thr = np.minimum(np.float32(a.epsilon), steps / np.float32(a.ramp))
        u = self.rng.next_blocks(B)   # one counter per row: batching-invariant
        exploit = u[:, 0] < thr
        out = np.minimum((u[:, 1] * 3.0).astype(np.int64), 2)
        if exploit.any():
            q = self.q_values(x[torch.from_numpy(exploit)]).cpu()
            out[exploit] = torch.argmax(q, dim=1).numpy()  # first max on ties, like TF ArgMax
        return out

    # ------------------------------------------------------------------ learning
    @property
    def last_loss(self) -> float:
        """Loss of the last update (read back from the GPU on first access)."""
        if self._loss_dev is not None:
            self._last_loss, self._loss_dev = float(self._loss_dev.sum()), None
        return self._last_loss

    def update(self, states: ArrayLike, rewards, next_states: ArrayLike, actions=None,
               return_loss: bool = True) -> Optional[float]:
        """One TD update over a batch (B=1 in the reference).  Returns the loss; with
        ``return_loss=False`` (the policy actor, which never reads it) the GPU path does not wait
        for the update to finish -- ``last_loss`` still reads it back on demand."""
        # host inputs stay on the host for the native path (one staged copy, F32Learner._stage)
        to = (lambda t: t) if self._k is not None else (lambda t: t.to(self.device))
        x = to(as_state(states, self.input_dim, "state"))
        xn = to(as_state(next_states, self.input_dim, "nextState"))
        if x.shape[0] != xn.shape[0]:
            raise IllegalArgumentException("state / nextState batch mismatch")
        B = x.shape[0]
        r = to(torch.from_numpy(np.broadcast_to(np.asarray(rewards, dtype=np.float32), (B,)).copy()))
        act = None
        if actions is not None:
            act = to(torch.from_numpy(np.broadcast_to(np.asarray(actions, dtype=np.int64), (B,)).copy()))
        a = self.cfg.agent
        compat = a.target_slot == "compat" or act is None
        coef = 2.0 / B if a.loss_reduction == "mean" else 2.0
        if self._k is not None:
            loss = self._k.td_update(x, r, xn, None if compat else act, coef, want_loss=return_loss)
        else:
            loss = self._torch_update(x, r, xn, None if compat else act, coef)
        self.iteration += 1
        if isinstance(loss, torch.Tensor):
            self._loss_dev = loss
            return None
        self._last_loss, self._loss_dev = loss, None
        return loss

    def _torch_update(self, x, r, xn, act, coef) -> float:
        L, a, m = self.layout, self.cfg.agent, self.cfg.model
        q, acts, xp = qn.forward(self.params, L, x, m.output_relu)
        qn_, _, _ = qn.forward(self.params, L, xn, m.output_relu)
        qa = qn_[:, : L.n_actions]
        nmax, amax = qa.max(dim=1)
        slot = amax if act is None else act
        target = r + np.float32(a.gamma) * (qa.gather(1, amax[:, None])[:, 0] if act is None else nmax)
        qs = q.gather(1, slot[:, None])[:, 0]
        diff = qs - target
        dq = torch.zeros_like(q)
        fb = diff.clamp(-a.td_clip, a.td_clip) if a.td_clip > 0 else diff   # Huber (agent.td_clip)
        dq.scatter_(1, slot[:, None], (coef * fb)[:, None])
        grad = qn.backward(self.params, L, xp, acts, q, dq, m.output_relu)
        qn.optimizer_step_ref(self.params, grad, self.opt, self.mask, a.lr, a.adam_betas, a.adam_eps)
        return float((diff * diff).sum())

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {
            "params": self.params.detach().cpu().clone(),
            "opt_s1": self.opt.s1.detach().cpu().clone(),
            "opt_s2": self.opt.s2.detach().cpu().clone(),
            "opt_t": torch.tensor([self.opt.t], dtype=torch.int64),
            "iteration": torch.tensor([self.iteration], dtype=torch.int64),
            "rng_counter": torch.tensor([self.rng.counter], dtype=torch.int64),
        }

    def load_state_dict(self, d: Dict[str, torch.Tensor]) -> None:
        self.params.copy_(d["params"].to(self.device))
        if self.opt.s1.numel():
            self.opt.s1.copy_(d["opt_s1"].to(self.device))
        if self.opt.s2.numel():
            self.opt.s2.copy_(d["opt_s2"].to(self.device))
        self.opt.t = int(d["opt_t"][0])
        self.iteration = int(d["iteration"][0])
        self.rng.counter = int(d["rng_counter"][0])
        if self._k is not None:
            self._k.sync_from_learner()
