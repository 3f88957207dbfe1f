#!/usr/bin/env python3
"""Overlapped-DP rehearsal on ONE GPU: the fused step kernel with k CUs held for T us per step.

In overlapped DP (engine.dp_overlap) RCCL's all-reduce of step t runs beside step t+1's fused
kernel, and every CU one of its workgroups holds cannot take a step-kernel workgroup (~159 KiB of
LDS each).  This tool stands a CU-occupying kernel (csrc/diag.hip ``st_occupy``: k workgroups x T us,
4 KiB LDS each) in for the collective, launched on a side stream just before each step, and times
the flagship step under the static and the dynamic chunk schedule (csrc/qstep_wide.hip).

    python tools/overlap_rehearsal.py --steps 100 -o gpurun_out/overlap.md
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(sched: str, k: int, usec: int, steps: int, warmup: int, envs: int) -> float:
    from sharetrade.config import preset_config
    from sharetrade.ops import native
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.envs_per_rank = envs
    cfg.engine.chunk_schedule = sched
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev)
    assert eng.chunk_schedule == sched, (eng.chunk_schedule, sched)
    L = native.lib()
    side = torch.cuda.Stream(dev)
    sink = torch.zeros(4096, dtype=torch.int32, device=dev)
    ev = torch.cuda.Event()

    def one():
        if k > 0:
            ev.record()
            side.wait_event(ev)
            native.check(L.st_occupy(k, usec, native.ptr(sink), side.cuda_stream), "occupy")
            # the overlapped step's update kernel sits between the collective's launch and the next
            # step kernel: a ~2 us spin on the main stream lets the stand-in dispatch first, as RCCL's does
            torch.cuda._sleep(4000)
        eng.step()

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--usec", type=int, default=25)
    ap.add_argument("--cus", default="0,8,32")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    import build as _b

    _b.build_all()
    rows = []
    for k in [int(x) for x in a.cus.split(",")]:
        r = {s: run(s, k, a.usec, a.steps, a.warmup, a.envs) for s in ("static", "dynamic")}
        rows.append((k, r["static"], r["dynamic"]))
        print(f"k={k:3d} CUs x {a.usec} us: static {r['static']:.4f} ms/step, dynamic {r['dynamic']:.4f} ms/step",
              flush=True)
    lines = [f"# Overlapped-DP rehearsal: fused step ({a.envs} envs) with k CUs held {a.usec} us per step",
             "", "| CUs held | static ms/step | dynamic ms/step | dynamic / static |", "|---|---|---|---|"]
    lines += [f"| {k} | {s:.4f} | {d:.4f} | {d / s:.3f} |" for k, s, d in rows]
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
