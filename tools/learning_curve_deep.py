#!/usr/bin/env python3
"""Does the config-4 learner learn?  4x1024-MLP replay DQN on the AR(1)-momentum price bank
(`data.source = "ar1"`): the trained run vs the same run with a frozen random network (lr = 0;
identical envs, draws and epsilon schedule), reward per env-step over windows of iterations.
Prints a markdown table (GPU)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def curve(lr: float, iters: int, window: int, envs: int):
    from sharetrade.config import preset_config
    from sharetrade.trainer.deep import DeepDQN

    cfg = preset_config("flagship")
    cfg.model.hidden = [1024, 1024, 1024, 1024]
    cfg.data.source = "ar1"
    cfg.agent.lr = lr
    d = DeepDQN(cfg, torch.device("cuda", 0), envs=envs, batch=4096, overlap_act=True)
    out = []
    prev_r, prev_steps = 0.0, 0
    d.capture()
    done = 1
    while done < iters:
        d.iteration()
        done += 1
        if done % window == 0:
            st = d.stats.detach().cpu().numpy().astype(np.float64)
            steps = d.env_steps * d.E
            out.append((done, (st[0] - prev_r) / max(1, steps - prev_steps)))
            prev_r, prev_steps = st[0], steps
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3000)
    ap.add_argument("--window", type=int, default=500)
    ap.add_argument("--envs", type=int, default=16384)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import build

    build.build_all()
    learned = curve(a.lr, a.iters, a.window, a.envs)
    frozen = curve(0.0, a.iters, a.window, a.envs)
    lines = ["# Config 4 learning check: 4x1024 MLP replay DQN on the AR(1)-momentum price bank (1x MI355X)", "",
             f"{a.envs} envs act per iteration, one update (batch 4,096 from the 1M-transition ring) per "
             f"iteration, lr {a.lr}; the frozen run has lr = 0 (same envs / draws / epsilon schedule).", "",
             "| iterations | reward / env-step (trained) | reward / env-step (frozen) |", "|---|---|---|"]
    for (i, r1), (_, r2) in zip(learned, frozen):
        lines.append(f"| {i - a.window + 1}-{i} | {r1:.4e} | {r2:.4e} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
