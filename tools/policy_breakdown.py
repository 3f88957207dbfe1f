#!/usr/bin/env python3
"""Where the flagship learner's greedy episode return comes from, vs random / buy-and-hold.

Trains the bench's engine exactly as ``bench.py`` does before its evaluation (flagship preset, the bench's envs
and bank, ``--train-steps`` Adam updates: 256 graph-priming + 5 warm-up + 20 timed = 281 by default), then plays
one full 5,846-step episode per env with each policy while recording, per env:

* the chosen actions (Buy / Sell / Hold shares) and the executed ones (shares actually moved);
* the shares held over each price interval s_{t-1} (the env's reward is s_{t-1} (v_t - v_{t-1}): a trade
  executes at the new price and changes no value by itself, so the episode return is sum_t s_{t-1} dv_t);
* the return split into EXPOSURE = mean(s) x (v_end - v_start) -- what holding the average position through
  the whole move earns -- and TIMING = return - exposure -- what varying the position earns;
* the correlation of the position with the price level (a rebalancer that holds less when the price is high
  has it negative).

Policies: greedy (learned, frozen, exploit-only), init_greedy (random-init net), random (uniform actions), and
"kelly" -- a fixed rule, not a learner: buy when the position is worth less than half the portfolio, else sell
(the log-optimal constant fraction of a zero-log-drift geometric walk, sigma^2 / 2 / sigma^2 = 1/2), to price
what a policy CAN reach on this bank's median.

Usage (GPU): python tools/policy_breakdown.py [--envs 1835008] [--train-steps 281] [--out profiles/x.md]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=7 << 18)
    ap.add_argument("--train-steps", type=int, default=281)
    ap.add_argument("--preset", default="flagship")
    ap.add_argument("--set", action="append", default=[], help="agent.KEY=VALUE overrides (floats / ints / str)")
    ap.add_argument("--policies", default="greedy,init_greedy,random,kelly,buy_hold")
    ap.add_argument("--out", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--cpu", action="store_true", help="plumbing check: torch backend on the CPU (tiny --envs)")
    a = ap.parse_args()

    if not a.cpu:
        import build

        build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    dev = torch.device("cpu") if a.cpu else torch.device("cuda", 0)
    cfg = preset_config(a.preset)
    cfg.engine.envs_per_rank = a.envs
    for kv in a.set:
        k, v = kv.split("=", 1)
        sec, key = k.split(".", 1)
        obj = getattr(cfg, sec)
        cur = getattr(obj, key)
        setattr(obj, key, type(cur)(v) if not isinstance(cur, bool) else v in ("1", "true", "True"))
    if a.cpu:
        cfg.engine.dtype = "fp32"
        cfg.data.length = 400
    eng = VectorEngine(cfg, device=dev, **({"backend": "torch", "envs": a.envs} if a.cpu else {}))
    init = eng.params.detach().clone()
    if not a.cpu:
        eng.capture_graph(warmup=0)
    eng.run(a.train_steps)
    eng.synchronize()
    H, T, E = int(eng.H), int(eng.T), eng.E
    steps = T - H
    P = eng.prices
    b0 = float(cfg.env.budget)
    res = {}

    def play(name, runner, engine=True):
        """runner(t) advances every env one step (pos == t for all envs: they start together)."""
        st = eng.state
        f64 = dict(dtype=torch.float64, device=dev)
        acts = torch.zeros(3, E, **f64)
        moved = torch.zeros(2, E, **f64)
        s_sum = torch.zeros(E, **f64)
        s_p = torch.zeros(E, **f64)
        p_sum = torch.zeros(E, **f64)
        p_sq = torch.zeros(E, **f64)
        s_sq = torch.zeros(E, **f64)
        ret = torch.zeros(E, **f64)
        zero_frac = torch.zeros(E, **f64)
        if engine:
            benchkit.reset_episodes(eng)
        s_prev = eng.state.shares.double().clone()
        v_prev = P[:, H].double().clone()   # the first step trades at P[:, H] with nothing held
        for t in range(steps):
            a_t = runner(t)
            v = P[:, t + H].double()
            # the interval (t-1, t] was held with s_prev
            if t > 0:
                ret += s_prev * (v - v_prev)
                s_sum += s_prev
                s_sq += s_prev * s_prev
                s_p += s_prev * v_prev
                p_sum += v_prev
                p_sq += v_prev * v_prev
                zero_frac += (s_prev == 0).double()
            if a_t is not None:
                acts.scatter_add_(0, a_t.long().view(1, -1), torch.ones(1, E, **f64))
            s_now = eng.state.shares.double() if t < steps - 1 else None
            if s_now is None:   # the last step resets the env: its post-trade shares are gone from the state
                break
            moved[0] += (s_now > s_prev).double()
            moved[1] += (s_now < s_prev).double()
            s_prev, v_prev = s_now, v
        n = steps - 1
        if engine:
            fin = eng.state.last_final.double() - b0
            # the env's own final portfolio (its fp32 arithmetic) vs the recorded decomposition
            chk = float((fin - ret).abs().max())
        else:
            fin, chk = ret, 0.0
        sm = s_sum / n
        vs, ve = P[:, H].double(), P[:, T - 1].double()
        expo = sm * (ve - vs)
        timing = ret - expo
        cov = s_p / n - sm * (p_sum / n)
        sd = ((s_sq / n - sm * sm).clamp_min(0) * (p_sq / n - (p_sum / n) ** 2).clamp_min(0)).sqrt()
        corr = torch.where(sd > 0, cov / sd, torch.zeros_like(sd))
        q = lambda x: float(x.float().median())   # noqa: E731
        r = {
            "mean": float(ret.mean()), "median": q(ret), "p10": float(ret.float().quantile(0.1)) if E <= 1 << 24 else None,
            "env_final_minus_sum_max_abs": chk,
            "act_buy": float(acts[0].mean() / steps), "act_sell": float(acts[1].mean() / steps),
            "act_hold": float(acts[2].mean() / steps),
            "moved_up": float(moved[0].mean() / n), "moved_down": float(moved[1].mean() / n),
            "mean_shares": float(sm.mean()), "median_mean_shares": q(sm), "zero_share_frac": float(zero_frac.mean() / n),
            "exposure_mean": float(expo.mean()), "exposure_median": q(expo),
            "timing_mean": float(timing.mean()), "timing_median": q(timing),
            "pos_price_corr_median": q(corr),
        }
        res[name] = r
        print(name, json.dumps(r), flush=True)

    pol = a.policies.split(",")
    with benchkit.evaluation_snapshot(eng):
        if "greedy" in pol:
            with eng.policy_overrides(epsilon=math.inf, lr=0.0):
                play("greedy", lambda t: (eng.step(), eng.actions().clone())[1])
        if "init_greedy" in pol:
            cur = eng.params.detach().clone()
            eng.set_params(init)
            with eng.policy_overrides(epsilon=math.inf, lr=0.0):
                play("init_greedy", lambda t: (eng.step(), eng.actions().clone())[1])
            eng.set_params(cur)
        if "random" in pol:
            with eng.policy_overrides(epsilon=0.0, lr=0.0):
                play("random", lambda t: (eng.step(), eng.actions().clone())[1])
    # the fixed-rule baselines on the same banks, in the env's own arithmetic (torch, fp32 like the kernel)
    st = eng.state

    def rule(name, decide):
        b = torch.full((E,), b0, dtype=torch.float32, device=dev)
        sh = torch.zeros(E, dtype=torch.int32, device=dev)

        class _S:   # a stand-in state for play()
            pass
        S = _S()
        S.shares = sh
        saved = eng.state
        eng.state = S

        def runner(t):
            nonlocal b, sh
            v = P[:, t + H]
            act = decide(b, sh, v)
            buy = (act == 0) & (b >= v)
            sell = (act == 1) & (sh > 0)
            b = torch.where(buy, b - v, torch.where(sell, b + v, b))
            sh = sh + buy.to(torch.int32) - sell.to(torch.int32)
            S.shares = sh
            return act
        try:
            play(name, runner, engine=False)
        finally:
            eng.state = saved

    if "kelly" in pol:
        rule("kelly", lambda b, sh, v: torch.where(sh.float() * v < 0.5 * (b + sh.float() * v),
                                                   torch.zeros_like(sh), torch.ones_like(sh)))
    if "buy_hold" in pol:
        rule("buy_hold", lambda b, sh, v: torch.zeros_like(sh))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"envs": E, "train_steps": a.train_steps, "preset": a.preset, "set": a.set, "policies": res}, f,
                      indent=1)
    if a.out:
        keys = ["mean", "median", "mean_shares", "zero_share_frac", "act_buy", "act_sell", "act_hold", "moved_up",
                "moved_down", "exposure_mean", "exposure_median", "timing_mean", "timing_median",
                "pos_price_corr_median"]
        lines = [f"# policy breakdown: {a.preset} {' '.join(a.set)}, {E} envs, {a.train_steps} training steps, "
                 f"one {steps}-step episode per env", "",
                 "| policy | " + " | ".join(keys) + " |", "|" + "---|" * (len(keys) + 1)]
        for k, r in res.items():
            lines.append(f"| {k} | " + " | ".join(f"{r[x]:.4g}" for x in keys) + " |")
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
