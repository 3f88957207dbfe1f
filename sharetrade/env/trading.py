"""Vectorised Buy/Sell/Hold trading environment + the engine-step oracle.

Reference environment (`TrainerChildActor.scala:82-146`), per worker, per step ``i``:

* state  = ``prices[i, i+201) ++ (budget, shares)``                      (:89-91)
* current portfolio = ``budget + shares * shareValue_prev`` (seed value 0.0) (:84-86, :92)
* trade price ``v = prices[i + 201]``                                      (:94)
* Buy if budget >= v: (budget - v, shares + 1); Sell if shares > 0:
  (budget + v, shares - 1); otherwise Hold (unchanged)                     (:118-123)
  — the reference evaluates these with the *constructor* budget/shares
  (quirk Q1, ``compat_decisions=True``), which makes every reward 0.
* reward = new portfolio - current portfolio; next state = window shifted by
  one ++ (budget', shares')                                                (:136-146)
* episode = ``N - 201`` steps; final portfolio ``b + s * v``               (:67-68)

:func:`engine_step_ref` is the plain-PyTorch/NumPy oracle of ONE fused engine
step for ``E`` environments (select -> env step -> TD target -> backward); the
fused HIP kernel (`csrc/qstep_fused.hip`) is tested against it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from ..models import qnet as qn
from ..utils import rng

FEATURES = {"raw": 0, "relative": 1}


@dataclass
class EnvState:
    """Per-env state, all length-E tensors (fp32 / int32)."""

    budget: torch.Tensor
    shares: torch.Tensor
    value: torch.Tensor      # previous trade price (seed 0.0, TrainerChildActor.scala:84-86)
    pos: torch.Tensor        # step index within the episode
    episodes: torch.Tensor   # completed episodes
    last_final: torch.Tensor  # final portfolio of the last completed episode
    ret_sum: torch.Tensor    # sum of rewards in the current episode

    @classmethod
    def create(cls, E: int, budget: float, shares: int, device="cpu") -> "EnvState":
        f = dict(dtype=torch.float32, device=device)
        i = dict(dtype=torch.int32, device=device)
        return cls(
            budget=torch.full((E,), float(budget), **f),
            shares=torch.full((E,), int(shares), **i),
            value=torch.zeros(E, **f),
            pos=torch.zeros(E, **i),
            episodes=torch.zeros(E, **i),
            last_final=torch.full((E,), float("nan"), **f),
            ret_sum=torch.zeros(E, **f),
        )

    def clone(self) -> "EnvState":
        return EnvState(*(getattr(self, k).clone() for k in self.__dataclass_fields__))

    def to(self, device) -> "EnvState":
        return EnvState(*(getattr(self, k).to(device) for k in self.__dataclass_fields__))

    def as_dict(self) -> Dict[str, torch.Tensor]:
        return {k: getattr(self, k) for k in self.__dataclass_fields__}


def features(windows: torch.Tensor, budget: torch.Tensor, shares: torch.Tensor, mode: str,
             budget0: float) -> torch.Tensor:
    """[E, H] price windows -> [E, H+2] state rows (fp32)."""
    E, H = windows.shape
    x = torch.empty(E, H + 2, dtype=torch.float32, device=windows.device)
    if mode == "raw":
        x[:, :H] = windows
        x[:, H] = budget
        x[:, H + 1] = shares.float()
    elif mode == "relative":
        last = windows[:, H - 1]
        inv = (1.0 / last).float()
        x[:, :H] = windows * inv[:, None] - 1.0
        ib0 = np.float32(1.0 / budget0)
        x[:, H] = budget * ib0
        x[:, H + 1] = (shares.float() * last) * ib0
    else:
        raise KeyError(mode)
    return x


def gather_windows(prices: torch.Tensor, pos: torch.Tensor, H: int, shift: int = 0) -> torch.Tensor:
    """Hankel gather ``prices[e, pos_e + shift : pos_e + shift + H]`` -> [E, H]."""
    E = prices.shape[0]
    idx = (pos.long() + shift)[:, None] + torch.arange(H, device=prices.device)[None, :]
    return torch.gather(prices, 1, idx)


def env_transition(a: torch.Tensor, b: torch.Tensor, s: torch.Tensor, v_prev: torch.Tensor,
                   v_new: torch.Tensor, compat: bool, b0: float, s0: int, relative: bool = False,
                   growth: bool = False):
    """Apply actions; returns (b', s', reward).  fp32 arithmetic, no FMA contraction.
    ``relative``: reward = change / previous portfolio value (0 where that value is not positive).
    ``growth`` (with ``relative``): reward = rel - rel^2 / 2, the portfolio's log growth log1p(rel) to second
    order -- its expectation is maximised by the Kelly fraction of wealth in the stock (mu / sigma^2: one half
    on a zero-log-drift geometric walk) instead of by the largest position (profiles/r6_policy_breakdown.md);
    the same three roundings as the kernels (rel * 0.5 exact, * rel, subtract)."""
    if compat:
        bd = torch.full_like(b, float(b0))
        sd = torch.full_like(s, int(s0))
    else:
        bd, sd = b, s
    buy = (a == 0) & (bd >= v_new)
    sell = (a == 1) & (sd > 0)
    b2 = torch.where(buy, bd - v_new, torch.where(sell, bd + v_new, bd))
    s2 = torch.where(buy, sd + 1, torch.where(sell, sd - 1, sd)).to(torch.int32)
    cur = b + s.float() * v_prev
    new = b2 + s2.float() * v_new
    r = new - cur
    if relative or growth:
        r = torch.where(cur > 0, r / torch.where(cur > 0, cur, torch.ones_like(cur)), torch.zeros_like(r))
    if growth:
        r = r - (r * 0.5) * r
    return b2, s2, r


def select_actions(q: torch.Tensor, pos: torch.Tensor, env_ids: np.ndarray, step: int, seed: int,
                   rank: int, epsilon: float, ramp: float, n_actions: int = 3):
    """Epsilon-greedy with the exploit ramp ``min(eps, i/ramp)`` (QDecisionPolicyActor.scala:58-62).
    ``epsilon = inf``: the greedy policy (exploit at every position, as the kernels' eps = inv_ramp = inf)."""
    u1, u2 = rng.uniforms(seed, rank, env_ids, step)
    if np.isinf(epsilon):
        thr = np.full(u1.shape, np.inf, dtype=np.float32)
    else:
        thr = np.minimum(np.float32(epsilon), pos.cpu().numpy().astype(np.float32) * np.float32(1.0 / ramp))
    exploit = torch.from_numpy(u1 < thr)
    greedy = torch.argmax(q[:, :n_actions].cpu(), dim=1)  # first max on ties (like TF ArgMax)
    rnd = torch.from_numpy(np.minimum((u2 * np.float32(n_actions)).astype(np.int64), n_actions - 1))
    a = torch.where(exploit, greedy, rnd).to(torch.int32)
    return a.to(q.device), exploit.to(q.device)


def engine_step_ref(prices: torch.Tensor, st: EnvState, params: torch.Tensor, layout: qn.QNetLayout, *,
                    history: int, feature_mode: str, budget0: float, shares0: int, compat_env: bool,
                    target_slot: str, gamma: float, output_relu: bool, epsilon: float, ramp: float,
                    seed: int, rank: int, step: int, loss_coef: float, env_offset: int = 0,
                    emulate_bf16: bool = False, forced_actions: Optional[torch.Tensor] = None,
                    reward_mode: str = "absolute", td_clip: float = 0.0,
                    target_params: Optional[torch.Tensor] = None, double_dqn: bool = False,
                    reward_scale: float = 1.0, ramp_pos: Optional[torch.Tensor] = None):
    """One fused engine step for all envs.  Returns ``(new_state, grad, info)``.

    ``loss_coef`` multiplies ``(q_slot - y)`` (2.0 for the reference's summed
    squared error, ``2/E_total`` for a batch mean).

    Learning-quality experiments (not in the reference, which bootstraps from the online net at the
    episode position's ramp, QDecisionPolicyActor.scala:58-71): ``target_params`` values Q(x') with a
    target copy of the parameters; ``double_dqn`` picks the max-Q(x') action with the online net and values
    it with the target; ``reward_scale`` multiplies the reward in the TD target; ``ramp_pos`` replaces the
    episode position in the exploit ramp (e.g. the global step count)."""
    E, T = prices.shape
    H = history
    pos = st.pos
    win = gather_windows(prices, pos, H)
    v_new = torch.gather(prices, 1, (pos.long() + H)[:, None])[:, 0]
    x = features(win, st.budget, st.shares, feature_mode, budget0)
    q, acts, xp = qn.forward(params, layout, x, output_relu, emulate_bf16)
    env_ids = np.arange(env_offset, env_offset + E, dtype=np.uint32)
    a, exploit = select_actions(q, pos if ramp_pos is None else ramp_pos, env_ids, step, seed, rank, epsilon, ramp,
                                layout.n_actions)
    if forced_actions is not None:
        a = forced_actions.to(torch.int32)
    b2, s2, r = env_transition(a, st.budget, st.shares, st.value, v_new, compat_env, budget0, shares0,
                               relative=(reward_mode in ("relative", "growth")), growth=(reward_mode == "growth"))
    win2 = gather_windows(prices, pos, H, shift=1)
    x2 = features(win2, b2, s2, feature_mode, budget0)
    q2, _, _ = qn.forward(params, layout, x2, output_relu, emulate_bf16)
    qa = q2[:, : layout.n_actions]
    qv = qa
    if target_params is not None:
        qt, _, _ = qn.forward(target_params, layout, x2, output_relu, emulate_bf16)
        qv = qt[:, : layout.n_actions]
    rs = r * reward_scale if reward_scale != 1.0 else r
    if target_slot == "compat":
        slot = torch.argmax(qa, dim=1)
        y = rs + gamma * qv.gather(1, slot[:, None])[:, 0]
    else:
        slot = a.long()
        if double_dqn:
            y = rs + gamma * qv.gather(1, torch.argmax(qa, dim=1)[:, None])[:, 0]
        else:
            y = rs + gamma * qv.max(dim=1).values
    qs = q.gather(1, slot[:, None])[:, 0]
    dq = torch.zeros_like(q)
    d = qs - y
    if td_clip > 0:
        d = d.clamp(-td_clip, td_clip)
    dq.scatter_(1, slot[:, None], (loss_coef * d)[:, None])
    grad = qn.backward(params, layout, xp, acts, q, dq, output_relu, emulate_bf16)
    loss = ((qs - y) ** 2).sum()

    ns = st.clone()
    ns.budget, ns.shares, ns.value = b2, s2, v_new.clone()
    ns.pos = pos + 1
    ns.ret_sum = st.ret_sum + r
    done = ns.pos >= (T - H)
    if bool(done.any()):
        final = b2 + s2.float() * v_new
        ns.last_final = torch.where(done, final, ns.last_final)
        ns.episodes = ns.episodes + done.int()
        ns.budget = torch.where(done, torch.full_like(b2, float(budget0)), ns.budget)
        ns.shares = torch.where(done, torch.full_like(s2, int(shares0)), ns.shares)
        ns.value = torch.where(done, torch.zeros_like(v_new), ns.value)
        ns.pos = torch.where(done, torch.zeros_like(ns.pos), ns.pos)
        ns.ret_sum = torch.where(done, torch.zeros_like(ns.ret_sum), ns.ret_sum)
    info = dict(q=q, q_next=q2, actions=a, reward=r, slot=slot, target=y, loss=loss, exploit=exploit,
                x=x, x_next=x2, dq=dq)
    return ns, grad, info
