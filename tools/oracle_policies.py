#!/usr/bin/env python3
"""What the trading env's action space lets a perfect-information policy earn (host simulation, NumPy).

The env trades ONE share per step (TrainerChildActor.scala:118-123, intended semantics: Buy if the budget
covers the price, Sell if a share is held).  On each bank this compares, over the same series:

* ``buy & hold``  -- Buy every step (the budget goes into shares at the start, then held);
* ``momentum 1``  -- Buy after an up day, Sell after a down day (the AR(1) bank's own signal, known exactly);
* ``momentum 50`` -- the same on the sign of the last 50 days' return (a trend follower);
* ``random``      -- uniform Buy / Sell / Hold.

Banks: ``ar1`` (log-return AR(1), phi 0.3, vol 0.02: the bank of tools/learning_curve.py) and ``trend``
(persistent zero-mean drift regimes, sharetrade.config.DataConfig.trend_*).  Reported: mean and median of
(final portfolio - budget) over the series.  Used in profiles/r4_learning_eval_65k.md.

    python tools/oracle_policies.py [--series 4000] [--length 6047]
"""
import argparse

import numpy as np


def bank(n, T, kind, phi=0.3, vol=0.02, rho=0.995, mu_sd=0.002, seed=1):
    g = np.random.default_rng(seed)
    r = np.zeros(n)
    lp = np.zeros(n)
    mu = g.normal(0.0, mu_sd, n)
    out = np.empty((n, T))
    out[:, 0] = 50.0
    for t in range(1, T):
        if kind == "ar1":
            r = phi * r + vol * g.standard_normal(n)
        else:
            mu = rho * mu + mu_sd * np.sqrt(1 - rho ** 2) * g.standard_normal(n)
            r = mu + vol * g.standard_normal(n)
        lp += r
        out[:, t] = 50.0 * np.exp(lp)
    return out.astype(np.float32)


def run(P, policy, H=201, b0=2400.0):
    n, T = P.shape
    b = np.full(n, b0, np.float32)
    s = np.zeros(n, np.int64)
    for pos in range(T - H):
        v = P[:, pos + H]
        a = policy(P, pos, H)
        buy = (a == 0) & (b >= v)
        sell = (a == 1) & (s > 0)
        b = np.where(buy, b - v, np.where(sell, b + v, b)).astype(np.float32)
        s = s + buy - sell
    return (b + s * P[:, -1]).astype(np.float64) - b0


def momentum(k):
    def pol(P, pos, H):
        r = np.log(P[:, pos + H - 1] / P[:, pos + H - 1 - k])
        return np.where(r > 0, 0, 1)
    return pol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=4000)
    ap.add_argument("--length", type=int, default=6047)
    a = ap.parse_args()
    rows = []
    for kind in ("ar1", "trend"):
        P = bank(a.series, a.length, kind)
        res = {"buy & hold": run(P, lambda P, pos, H: np.zeros(P.shape[0], int)),
               "momentum 1": run(P, momentum(1)), "momentum 50": run(P, momentum(50)),
               "random": run(P, lambda P, pos, H: np.random.default_rng(pos).integers(0, 3, P.shape[0]))}
        for k, v in res.items():
            rows.append(f"| {kind} | {k} | {v.mean():.0f} | {np.median(v):.0f} |")
    print(f"# One-share-per-step policies with perfect information ({a.series} series x {a.length - 201} steps)\n")
    print("| bank | policy | mean | median |\n|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
