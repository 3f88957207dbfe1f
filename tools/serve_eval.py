#!/usr/bin/env python3
"""Train -> serve -> trade on unseen prices: the served flagship policy out of sample.

1. Train the flagship online DQN (``VectorEngine``, fused HIP step kernel) on an AR(1)-momentum price
   bank (``data.source = "ar1"``; a plain random walk has nothing to learn).
2. Hand its weights to a :class:`sharetrade.serve.PolicyServer` (``csrc/qserve.hip``).
3. Trade one full episode on a bank generated with a different seed (never seen in training): at each
   day every env sends its ``SelectionAction`` row (201 prices, budget, shares) and the server answers
   the whole batch with one launch (greedy); the Buy/Sell/Hold transition is
   ``sharetrade.env.trading.env_transition`` (the intended semantics, ``TrainerChildActor.scala:118-146``
   with quirk Q1 fixed).

Reported per policy: mean / population std of the final portfolios (the reference's ``GetAvg`` /
``GetStd``, ``TrainerRouterActor.scala:148-151``), for the trained net, the same net untrained, a
uniform random policy and buy-and-hold.

    python tools/serve_eval.py --train-steps 12000 --envs 65536 --eval-envs 8192 -o profiles/r2_serve_eval.md
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trade(prices: torch.Tensor, H: int, budget0: float, policy) -> torch.Tensor:
    """One episode over every row of ``prices`` [E, T]; returns the final portfolios [E] (fp64)."""
    from sharetrade.env import trading as tr

    E, T = prices.shape
    dev = prices.device
    b = torch.full((E,), float(budget0), device=dev)
    s = torch.zeros(E, dtype=torch.int32, device=dev)
    v = prices[:, H - 1].clone()
    for t in range(T - H):
        rows = torch.cat([prices[:, t:t + H], b[:, None], s[:, None].float()], 1)
        a = policy(rows, t)
        v_new = prices[:, t + H]
        b, s, _ = tr.env_transition(a, b, s, v, v_new, compat=False, b0=budget0, s0=0)
        v = v_new
    return (b.double() + s.double() * v.double())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=12000)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--eval-envs", type=int, default=8192)
    ap.add_argument("--phi", type=float, default=0.3)
    ap.add_argument("--ema-decay", type=float, default=0.999, help="engine.ema_decay: also serve the Polyak average")
    ap.add_argument("-o", "--out", default=None)
    args = ap.parse_args()

    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.models import qnet as qn
    from sharetrade.serve import PolicyServer
    from sharetrade.trainer.engine import VectorEngine, make_price_bank

    dev = torch.device("cuda", 0)
    cfg = preset_config("flagship")
    cfg.data.source = "ar1"
    cfg.data.ar_phi = args.phi
    cfg.engine.ema_decay = args.ema_decay
    H, b0 = cfg.model.history, cfg.env.budget

    t0 = time.perf_counter()
    eng = VectorEngine(cfg, device=dev, envs=args.envs)
    eng.capture_graph(warmup=0)
    eng.run(args.train_steps)
    eng.synchronize()
    train_s = time.perf_counter() - t0
    st = eng.stats_dict()

    test = make_price_bank(cfg, args.eval_envs, dev, seed=101)   # another seed: unseen series
    trained = PolicyServer(cfg, params=eng.params, device=dev, backend="native")
    averaged = PolicyServer(cfg, params=eng.serving_params, device=dev, backend="native")
    untrained = PolicyServer(cfg, params=qn.init_params(trained.layout, cfg.model, seed=cfg.agent.seed), device=dev,
                             backend="native")
    g = torch.Generator(device=dev)
    g.manual_seed(5)

    def served(srv):
        return lambda rows, t: srv.infer(rows).long()

    def served_eps(srv):   # the reference's SelectionAction semantics: step = the day index (exploit ramp)
        return lambda rows, t: srv.infer(rows, torch.full((rows.shape[0],), float(t), device=dev)).long()

    def rand(rows, t):
        return torch.randint(0, 3, (rows.shape[0],), device=dev, generator=g)

    def hold_after_buy(rows, t):   # buy-and-hold: buy on day one, hold after
        return torch.full((rows.shape[0],), 0 if t == 0 else 2, device=dev, dtype=torch.long)

    res = {}
    pols = [("trained net, greedy (served)", served(trained))]
    if args.ema_decay > 0:
        pols.append((f"Polyak average (decay {args.ema_decay}), greedy (served)", served(averaged)))
    pols += [("trained net, epsilon-greedy as in training (served)", served_eps(trained)),
             ("untrained net, greedy (served)", served(untrained)),
             ("uniform random", rand), ("buy one share, hold", hold_after_buy)]
    for name, pol in pols:
        t1 = time.perf_counter()
        f = trade(test, H, b0, pol)
        torch.cuda.synchronize()
        res[name] = {"mean": float(f.mean()), "std": float(f.std(unbiased=False)), "median": float(f.median()),
                     "return_pct": float((f.mean() / b0 - 1) * 100), "seconds": round(time.perf_counter() - t1, 2)}
        print(name, json.dumps(res[name]), flush=True)

    # the same greedy policy on series it was trained on (in sample): overfitting vs the exploration mix
    t1 = time.perf_counter()
    f = trade(eng.prices[: args.eval_envs], H, b0, served(trained))
    torch.cuda.synchronize()
    res["trained net, greedy, on training series (in sample)"] = {
        "mean": float(f.mean()), "std": float(f.std(unbiased=False)), "median": float(f.median()),
        "return_pct": float((f.mean() / b0 - 1) * 100), "seconds": round(time.perf_counter() - t1, 2)}
    days = test.shape[1] - H
    lines = [
        "# Train -> serve -> trade on unseen prices (`tools/serve_eval.py`, 1x MI355X)",
        "",
        f"Training: flagship online DQN, {args.envs:,} envs x {args.train_steps:,} steps on an AR(1)-momentum bank "
        f"(phi {args.phi}), {train_s:.1f} s including bank generation and graph capture; in sample, "
        f"{st['episodes_done']:,.0f} finished episodes ended at a mean portfolio of "
        f"{st['final_sum'] / max(st['episodes_done'], 1):,.0f}.",
        "",
        f"Evaluation: {args.eval_envs:,} unseen series (bank seed 101), one episode of {days:,} days from budget "
        f"{b0:,.0f}; every day one batched `SelectionAction` launch for all envs (greedy, or epsilon-greedy with "
        f"the training schedule: exploit probability min({cfg.agent.epsilon}, day / {cfg.agent.ramp:g})).",
        "",
        "| policy | mean final portfolio (GetAvg) | std (GetStd) | median | mean return | seconds |",
        "|---|---|---|---|---|---|",
    ]
    for name, r in res.items():
        lines.append(f"| {name} | {r['mean']:,.1f} | {r['std']:,.1f} | {r['median']:,.1f} | {r['return_pct']:+.1f} % | "
                     f"{r['seconds']} |")
    tg, rd = res["trained net, greedy (served)"], res["uniform random"]
    lines += ["", f"Greedy trained vs uniform random out of sample: mean {tg['mean']:,.0f} vs {rd['mean']:,.0f}, "
              f"median {tg['median']:,.0f} vs {rd['median']:,.0f} (std >> mean: compounding on the momentum series "
              "gives a heavy right tail)."]
    txt = "\n".join(lines) + "\n"
    print(txt)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
