#!/usr/bin/env python3
"""Does the config-5 learner learn?  GRU(256) DQN on synthetic minute bars (AR(1) + GARCH returns,
trading cost per position change): the trained run vs the same run with a frozen random network
(lr = 0; identical envs, draws and epsilon schedule), reward per env-step over windows of
iterations.  Prints a markdown table (GPU)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def curve(lr: float, iters: int, window: int, envs: int, seed: int):
    from sharetrade.config import preset_config
    from sharetrade.trainer.recurrent import RecurrentDQN

    cfg = preset_config("recurrent")
    d = RecurrentDQN(cfg, torch.device("cuda", 0), envs=envs, lr=lr, seed=seed, overlap_act=True)
    out = []
    prev_r, prev_steps, prev_ep, prev_fin = 0.0, 0, 0.0, 0.0
    d.capture()
    done = 1
    while done < iters:
        d.iteration(1)
        done += 1
        if done % window == 0:
            st = d.stats.detach().cpu().numpy().astype(np.float64)
            steps = d.env_steps
            r = (st[0] - prev_r) / max(1, steps - prev_steps)
            ep = st[2] - prev_ep
            ret = (st[3] - prev_fin) / ep if ep > 0 else float("nan")
            out.append((done, r, ret, 1.0 - (st[1] - 0) / max(1, steps)))
            prev_r, prev_steps, prev_ep, prev_fin = st[0], steps, st[2], st[3]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=1500)
    ap.add_argument("--window", type=int, default=250)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import build

    build.build_all()
    learned = curve(3e-4, a.iters, a.window, a.envs, a.seed)
    frozen = curve(0.0, a.iters, a.window, a.envs, a.seed)
    lines = ["# Config 5 learning check: GRU(256) DQN on AR(1)+GARCH minute bars (1x MI355X)", "",
             f"{a.envs} envs x 16 bars per iteration, one update (1,024 segments) per iteration; the frozen run "
             "has lr = 0 (random-init network, same envs / draws / epsilon schedule).", "",
             "| iterations | reward / env-step (trained) | reward / env-step (frozen) | episode return (trained) | "
             "episode return (frozen) |", "|---|---|---|---|---|"]
    for (i, r1, e1, _), (_, r2, e2, _) in zip(learned, frozen):
        lines.append(f"| {i - a.window + 1}-{i} | {r1:.3e} | {r2:.3e} | {e1:.4f} | {e2:.4f} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
