"""``tools/serve_eval.py``'s episode simulator (CPU): closed-form checks of the trading loop the
train -> serve -> trade evaluation (profiles/r2_serve_eval.md) reports."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _prices(E=3, T=40):
    t = torch.arange(T, dtype=torch.float32)
    return torch.stack([10.0 + t, 50.0 - 0.5 * t, 20.0 + 0.0 * t])[:E]


def test_buy_one_share_and_hold_is_closed_form():
    from serve_eval import trade

    H, b0 = 5, 100.0
    p = _prices()
    f = trade(p, H, b0, lambda rows, t: torch.full((rows.shape[0],), 0 if t == 0 else 2, dtype=torch.long))
    want = b0 - p[:, H].double() + p[:, -1].double()   # buy at the first trade price, hold to the end
    assert torch.allclose(f, want)


def test_always_hold_keeps_the_budget_and_rows_are_state_layout():
    from serve_eval import trade

    H, b0 = 5, 100.0
    p = _prices()
    seen = []

    def hold(rows, t):
        seen.append(rows.clone())
        return torch.full((rows.shape[0],), 2, dtype=torch.long)

    f = trade(p, H, b0, hold)
    assert torch.equal(f, torch.full((3,), b0, dtype=torch.float64))
    assert len(seen) == p.shape[1] - H
    r0 = seen[3]   # day 3: prices t..t+H-1, then budget, then shares (TrainerChildActor.scala:90-91)
    assert torch.equal(r0[:, :H], p[:, 3:3 + H]) and torch.equal(r0[:, H], torch.full((3,), b0))
    assert torch.equal(r0[:, H + 1], torch.zeros(3))


def test_buy_every_day_spends_until_broke():
    from serve_eval import trade

    H, b0 = 5, 100.0
    p = _prices(E=1)
    f = trade(p, H, b0, lambda rows, t: torch.zeros(rows.shape[0], dtype=torch.long))
    assert 0.0 <= float(f[0]) and float(f[0]) >= b0 - 1e-3   # price only rises: value never below budget
