#!/usr/bin/env python3
"""Does the flagship engine learn?  Mean reward per env-step over training on a learnable series.

A plain random walk (the bench's data) has no predictable structure, so any policy earns ~0 in
expectation.  Here the price bank is an AR(1)-momentum walk (``data.source = "ar1"``: log-return
autocorrelation phi), and three runs share bank, seed and schedule:

* ``learned``  -- the flagship online DQN (epsilon-greedy ramp, Adam, TD update every step);
* ``random``   -- epsilon = 0: the exploit probability min(eps, pos/ramp) is 0, every action uniform;
* ``frozen``   -- the same epsilon-greedy schedule with lr = 0 (greedy w.r.t. the random-init net).

    python tools/learning_curve.py --steps 30000 --envs 65536 -o gpurun_out/learning.md
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(kind: str, steps: int, envs: int, every: int, phi: float, device: torch.device, sets=()):
    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine
    from sharetrade.utils.metrics import WindowStats

    cfg = preset_config("flagship")
    cfg.data.source = "ar1"
    cfg.data.ar_phi = phi
    cfg.override(list(sets))
    if kind == "random":
        cfg.agent.epsilon = 0.0
    if kind == "frozen":
        cfg.agent.lr = 0.0
    eng = VectorEngine(cfg, device=device, envs=envs)
    if eng.backend == "native" and device.type == "cuda":
        eng.capture_graph(warmup=0)
    ws = WindowStats()
    ws.window(eng.stats_dict(), eng.step_count, eng.E)
    rows = []
    while eng.step_count < steps:
        eng.step()
        if eng.step_count % every == 0:
            eng.synchronize()
            r = ws.window(eng.stats_dict(), eng.step_count, eng.E)
            rows.append(r)
            print(kind, json.dumps({k: round(v, 5) if isinstance(v, float) else v for k, v in r.items()}),
                  flush=True)
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30000)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--every", type=int, default=1000)
    ap.add_argument("--phi", type=float, default=0.3)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--set", action="append", default=[], help="config override section.key=value")
    ap.add_argument("--kinds", default="learned,random,frozen")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    if a.device == "cuda":
        import build as _b

        _b.build_all()
    dev = torch.device(a.device)
    kinds = a.kinds.split(",")
    res = {k: run(k, a.steps, a.envs, a.every, a.phi, dev, a.set) for k in kinds}
    lines = [f"# Learning curve: flagship online DQN (2x128 MLP, bf16 fused step) on an AR(1)-momentum "
             f"price bank (phi = {a.phi}, vol 0.02, 6,047 days), {a.envs} envs", "",
             "Reward = the portfolio's one-step return (`agent.reward_mode = relative`, flagship preset), "
             f"mean per env-step in basis points, per window of {a.every} steps; same bank and seed for every "
             "run (`tools/learning_curve.py`).  All envs start together, so every env ends an "
             "episode (5,846 steps) in the same window: the final-portfolio columns (budget 2,400 at the "
             "start of each episode) are filled there." + (f"  Overrides: {' '.join(a.set)}." if a.set else ""), ""]
    head = ["step"] + [f"{k} bp/step" for k in kinds] + [f"{k} final $" for k in kinds]
    if "learned" in kinds:
        head += ["learned TD loss", "learned explore"]
    lines += ["| " + " | ".join(head) + " |", "|" + "---|" * len(head)]
    fp = lambda r: f"{r['final_portfolio_mean']:.1f}" if "final_portfolio_mean" in r else ""
    for i, r0 in enumerate(res[kinds[0]]):
        rows = [res[k][i] for k in kinds]
        cells = [str(r0["step"])] + [f"{r['mean_reward'] * 1e4:.3f}" for r in rows] + [fp(r) for r in rows]
        if "learned" in kinds:
            rl = res["learned"][i]
            cells += [f"{rl['mean_td_loss']:.2e}", f"{rl['explore_rate']:.3f}"]
        lines.append("| " + " | ".join(cells) + " |")
    for k in kinds:
        m = sum(r["mean_reward"] for r in res[k]) / max(1, len(res[k]))
        lines.append(f"\n{k}: mean {m * 1e4:.3f} bp per env-step over {a.steps} steps")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
