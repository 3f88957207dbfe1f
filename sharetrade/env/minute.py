"""Minute-bar trading env (BASELINE config 5) — host reference of the env step fused into
``csrc/gru.hip::gru_act_kernel``.

Semantics (a per-bar version of the reference's Buy/Sell/Hold decisions,
`TrainerChildActor.scala:118-123`, with one share like its ``shares`` counter):

* action 0 Buy -> long 1 unit (entry = close_t when opening), 1 Sell -> flat, 2 Hold -> keep;
* reward = position' * ret_t - cost * [position changed], ret_t = (close_{t+1} / close_t - 1) * 100
  precomputed per bar (``data.minute_bars.bar_returns``);
* an episode is ``ep_len`` bars from a random start; on the last bar the env resets to a new
  Philox-drawn start, flat, and the recurrent state restarts from zero;
* exploration: exploit with probability ``min(eps, step * inv_ramp)`` (``step`` = global actor
  step), else a uniform random action (QDecisionPolicyActor.scala:56-62 with a global ramp).

All arithmetic is float32 in the same order as the kernel, so with random actions the
host and device trajectories agree bit for bit.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..utils import rng

TAG_ACT = 0x47525531  # "GRU1"
f32 = np.float32


@dataclass
class MinuteEnvState:
    t: int
    es: int
    pz: int = 0
    entry: float = 0.0
    ep_ret: float = 0.0
    episodes: int = 0


def obs(feat_row: np.ndarray, close_t: float, st: MinuteEnvState, ep_len: int) -> np.ndarray:
    """x_t (32 floats): 8 market features, position, unrealised pnl %, elapsed fraction, 1, zeros."""
    x = np.zeros(32, np.float32)
    x[:8] = feat_row
    x[8] = f32(st.pz)
    x[9] = (f32(close_t) / f32(st.entry) - f32(1)) * f32(100) if st.pz else f32(0)
    x[10] = f32(st.t - st.es) * f32(1.0 / ep_len)
    x[11] = f32(1)
    return x


def draws(env: int, step: int, key0, key1):
    """The actor's Philox draws for (env, global step): (explore coin, random action, reset start u)."""
    c0, c1, c2, _ = rng.philox4x32(np.uint32(env), np.uint32(step & 0xFFFFFFFF), np.uint32(step >> 32),
                                   np.uint32(TAG_ACT), key0, key1)
    return rng.u24(c0), rng.u24(c1), rng.u24(c2)


def step(st: MinuteEnvState, a: int, close: np.ndarray, ret: np.ndarray, T: int, ep_len: int, cost: float,
         u_reset: float):
    """Apply action ``a`` at bar ``st.t`` in place; returns (reward, done, finished-episode return)."""
    c_t = f32(close[st.t])
    np_ = 1 if a == 0 else (0 if a == 1 else st.pz)
    trade = np_ != st.pz
    if trade and np_ == 1:
        st.entry = float(c_t)
    rew = f32(np_) * f32(ret[st.t]) - (f32(cost) if trade else f32(0))
    st.ep_ret = float(f32(st.ep_ret) + rew)
    t1 = st.t + 1
    done = (t1 - st.es) >= ep_len
    fin = None
    if done:
        st.episodes += 1
        fin = st.ep_ret
        st.es = min(int(f32(u_reset) * f32(T - ep_len - 1)), T - ep_len - 2)
        t1 = st.es
        st.pz = 0
        st.ep_ret = 0.0
    else:
        st.pz = np_
    st.t = t1
    return float(rew), done, fin
