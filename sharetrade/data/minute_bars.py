"""Synthetic minute bars for the recurrent agent (BASELINE config 5).

The reference only ever trades a daily close series (`SharePriceGetter.scala:83-102`,
MSFT CSV); config 5 asks for a GRU on *minute-bar sequences*, and there is no network
for real intraday data, so bars are synthesised per env:

* log return  ``r_t = phi * r_{t-1} + sig_t * n1``  (AR(1): a weak, learnable momentum edge)
* variance    ``var_{t+1} = omega + alpha (r_t / u_t)^2 + beta var_t``  (GARCH(1,1) on the
  de-seasonalised return: volatility clusters)
* intraday    ``sig_t = sqrt(var_t) * u_t``, ``u_t = 1 + 0.8 x^2``, x = time-of-day in [-1, 1) (U-shape)
* OHLC: open = previous close, high/low = max/min(open, close) * exp(+-0.5 sig |n|), volume
  lognormal with the same U-shape.

Eight features per bar (bf16 on the GPU): return %, high-low range %, close position in the
bar's range, log volume, sin/cos time-of-day, 5-bar momentum %, current sigma %.

``generate_numpy`` is the host reference of ``csrc/gru.hip::minute_bars_kernel`` (same
Philox counters, same float32 formulas; transcendental ULPs differ, so parity is to
~1e-4 relative) and ``generate_gpu`` runs the kernel.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np
import torch

from ..utils import rng

NFEAT = 8
TAG = 0x4D424152  # "MBAR"


@dataclass
class BarParams:
    day: int = 390          # bars per session
    sigma: float = 1e-3     # per-minute volatility (long-run)
    phi: float = 0.08       # AR(1) coefficient of returns
    alpha: float = 0.05     # GARCH
    beta: float = 0.90
    p0: float = 100.0       # starting price scale (x U[0.5, 1.5))


def generate_numpy(E: int, T: int, bp: BarParams = BarParams(), seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """(close [E, T] float32, feat [E, T, 8] float32) — float32 host reference of the kernel."""
    f = np.float32
    k0, k1 = rng.key_for(seed, 0)
    e = np.arange(E, dtype=np.uint32)
    c0, _, _, _ = rng.philox4x32(e, np.full(E, 0xFFFFFFFF, np.uint32), np.zeros(E, np.uint32),
                                 np.full(E, TAG, np.uint32), k0, k1)
    c = f(bp.p0) * (f(0.5) + rng.u24(c0))
    var = np.full(E, f(bp.sigma) * f(bp.sigma), np.float32)
    rprev = np.zeros(E, np.float32)
    omega = f(bp.sigma) * f(bp.sigma) * (f(1) - f(bp.alpha) - f(bp.beta))
    hist = np.zeros((4, E), np.float32)
    close = np.zeros((E, T), np.float32)
    feat = np.zeros((E, T, NFEAT), np.float32)
    twopi = f(6.2831853)
    for t in range(T):
        a0, a1, a2, a3 = rng.philox4x32(e, np.full(E, t, np.uint32), np.zeros(E, np.uint32),
                                        np.full(E, TAG, np.uint32), k0, k1)
        u0 = np.maximum(rng.u24(a0), f(1e-7))
        u1 = rng.u24(a1)
        u2 = np.maximum(rng.u24(a2), f(1e-7))
        u3 = rng.u24(a3)
        rad0 = np.sqrt(f(-2) * np.log(u0)).astype(np.float32)
        rad1 = np.sqrt(f(-2) * np.log(u2)).astype(np.float32)
        n1 = rad0 * np.cos(twopi * u1).astype(np.float32)
        n2 = rad0 * np.sin(twopi * u1).astype(np.float32)
        n3 = rad1 * np.cos(twopi * u3).astype(np.float32)
        n4 = rad1 * np.sin(twopi * u3).astype(np.float32)
        tod = t % bp.day
        x = f(2) * f(tod) / f(bp.day) - f(1)
        ush = f(1) + f(0.8) * x * x
        sig = np.sqrt(var).astype(np.float32) * ush
        ret = f(bp.phi) * rprev + sig * n1
        opn = c
        c = (opn * np.exp(ret)).astype(np.float32)
        hi = np.maximum(opn, c) * np.exp(f(0.5) * sig * np.abs(n2)).astype(np.float32)
        lo = np.minimum(opn, c) * np.exp(f(-0.5) * sig * np.abs(n3)).astype(np.float32)
        vol = np.exp(f(0.5) * n4).astype(np.float32) * ush
        dsr = ret / ush
        var = omega + f(bp.alpha) * dsr * dsr + f(bp.beta) * var
        mom = ret + hist[0] + hist[1] + hist[2] + hist[3]
        hist[3], hist[2], hist[1], hist[0] = hist[2], hist[1], hist[0], ret
        rprev = ret
        ang = twopi * f(tod) / f(bp.day)
        close[:, t] = c
        feat[:, t, 0] = ret * f(100)
        feat[:, t, 1] = (hi - lo) / c * f(100)
        feat[:, t, 2] = (c - lo) / np.maximum(hi - lo, f(1e-12)) - f(0.5)
        feat[:, t, 3] = np.log(vol)
        feat[:, t, 4] = np.sin(ang)
        feat[:, t, 5] = np.cos(ang)
        feat[:, t, 6] = mom * f(100)
        feat[:, t, 7] = sig * f(100)
    return close, feat


def generate_gpu(E: int, T: int, device: torch.device, bp: BarParams = BarParams(), seed: int = 0):
    """(close [E, T] fp32, feat [E, T, 8] bf16) on the GPU (csrc/gru.hip minute_bars_kernel)."""
    from ..ops import gru as G
    from ..ops import native

    close = torch.empty(E, T, dtype=torch.float32, device=device)
    feat = torch.empty(E, T, NFEAT, dtype=torch.bfloat16, device=device)
    k0, k1 = (int(x) for x in rng.key_for(seed, 0))
    a = G.MinuteBarsArgs(close.data_ptr(), feat.data_ptr(), E, T, bp.day, bp.sigma, bp.phi, bp.alpha, bp.beta,
                         bp.p0, k0, k1)
    native.check(G.lib().st_minute_bars(a, native.stream_handle()), "st_minute_bars")
    return close, feat


def bar_returns(close):
    """ret[:, t] = (close[:, t+1] / close[:, t] - 1) * 100 (float32, last bar 0) -- the env's
    per-bar reward of a long unit, precomputed once so the actor's env step has no division."""
    if isinstance(close, np.ndarray):
        r = np.zeros_like(close, dtype=np.float32)
        r[:, :-1] = (close[:, 1:] / close[:, :-1] - np.float32(1)) * np.float32(100)
        return r
    r = torch.zeros_like(close)
    r[:, :-1] = (close[:, 1:] / close[:, :-1] - 1.0) * 100.0
    return r
