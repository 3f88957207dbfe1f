"""tools/oracle_policies.py: the one-share-per-step policy simulator behind profiles/r4_oracle_policies.md
(why buy-and-hold's mean return is out of reach for one-share trading on the geometric banks)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import oracle_policies as op  # noqa: E402


def _hold(P, pos, H):
    return np.zeros(P.shape[0], int)


def test_buy_and_hold_on_a_rising_line_buys_what_the_budget_covers():
    T, H = 260, 201
    P = np.tile(np.linspace(10.0, 20.0, T, dtype=np.float32), (3, 1))
    out = op.run(P, _hold, H=H, b0=100.0)
    # Buy every step: shares whenever the budget covers the price, then held to the last price
    b, s = 100.0, 0
    for pos in range(T - H):
        v = float(P[0, pos + H])
        if b >= v:
            b, s = b - v, s + 1
    assert np.allclose(out, b + s * float(P[0, -1]) - 100.0, rtol=1e-5)


def test_momentum_oracle_and_random_run_on_both_banks():
    for kind in ("ar1", "trend"):
        P = op.bank(64, 400, kind, seed=3)
        assert P.shape == (64, 400) and np.all(P > 0)
        for pol in (op.momentum(1), op.momentum(50)):
            r = op.run(P, pol)
            assert r.shape == (64,) and np.all(np.isfinite(r))
