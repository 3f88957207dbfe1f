#!/usr/bin/env python3
"""Per-step time of the flagship step after an idle gap (GPU events around every step).

Runs the bench configuration (1M envs), warms up, then for each idle gap: host sync, sleep, and
20 single-step graph replays timed individually.  Shows how long the slowdown after the bench's
host-side synchronisation lasts and whether it depends on the length of the idle gap.
Usage (GPU): python tools/dvfs_probe.py [--envs N] [--out profiles/x.md]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.envs_per_rank = a.envs
    eng = VectorEngine(cfg, device=torch.device("cuda", 0))
    eng.capture_graph(warmup=2, prime=True)
    eng.run(200)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    lines = [f"# step time after an idle gap ({a.envs} envs, single-step graph replays, GPU events)\n",
             "| idle gap | " + " | ".join(f"s{i}" for i in range(a.steps)) + " | mean |",
             "|---|" + "---|" * (a.steps + 1)]
    for gap in (0.0, 0.0001, 0.001, 0.01, 0.1, 0.0):
        torch.cuda.synchronize()
        if gap:
            time.sleep(gap)
        ev[0].record()
        for i in range(a.steps):
            eng.step()
            ev[i + 1].record()
        torch.cuda.synchronize()
        t = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.steps)]
        lines.append(f"| {gap * 1e3:g} ms | " + " | ".join(f"{x:.0f}" for x in t) + f" | {sum(t) / len(t):.0f} |")
        print(lines[-1], flush=True)
    # back-to-back without any sync, for reference
    ev[0].record()
    for i in range(a.steps):
        eng.step()
        ev[i + 1].record()
    eng.run(100)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.steps)]
    lines.append("| none (continued) | " + " | ".join(f"{x:.0f}" for x in t) + f" | {sum(t) / len(t):.0f} |")
    txt = "\n".join(lines) + "\n(us per step)\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
