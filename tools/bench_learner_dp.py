#!/usr/bin/env python3
"""What the data-parallel code path costs the config-4 / config-5 learners on ONE GPU (wire time
excluded): the DP path runs over a one-rank RCCL group with world_size forced to 2 (the all-reduce is
a real RCCL launch of the whole gradient, its result the rank's own gradient).  Modes: ``single``
(no DP), ``split`` (all-reduce between two captured graphs), ``ingraph`` (all-reduce captured in the
update graph; config 4: per layer on a comm stream beside the backward).  Prints one markdown table."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(kind, mode, iters, warm, ctx):
    from sharetrade.config import preset_config
    from sharetrade.trainer.runs import build, run

    cfg = preset_config("flagship" if kind == "deep" else "recurrent")
    kw = {"hidden": [1024] * 4} if kind == "deep" else {}
    dev = torch.device("cuda", 0)
    if mode in ("single", "single_unfused"):
        if mode == "single_unfused":
            kw["fused_adam"] = False
        d = build(kind, cfg, dev, **kw)
        run(kind, cfg, warm, device=dev, learner=d, log_every=0)
    else:
        d = build(kind, cfg, dev, world_size=2, **kw)
        run(kind, cfg, warm, device=dev, learner=d, ctx=ctx, capture_sync=mode.startswith("ingraph"),
            layer_overlap=(mode == "ingraph"), log_every=0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        d.iteration(1)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    del d
    torch.cuda.empty_cache()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    import torch.distributed as dist

    import build as B
    from sharetrade.parallel.dist import DistContext

    B.build_all()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ctx = DistContext(0, 2, 0, "nccl", dev, dist.group.WORLD)
    rows = ["# DP code path on one GPU (one-rank RCCL group, world_size forced to 2; wire time excluded)", "",
            f"{a.iters} timed iterations after {a.warmup} (graph capture included in the warm-up).", "",
            "| learner | single GPU (ms/iter) | single GPU, per-layer Adam + bias row sums | DP, all-reduce between "
            "graphs | DP, one all-reduce in the graph | DP, per-layer all-reduce on a comm stream |",
            "|---|---|---|---|---|---|"]
    for kind, name in (("deep", "config 4 (4x1024 MLP, batch 4096)"), ("recurrent", "config 5 (GRU(256))")):
        modes = ("single", "single_unfused", "split", "ingraph_flat", "ingraph")
        t = {m: (_time(kind, m, a.iters, a.warmup, ctx) if kind == "deep" or m in ("single", "split", "ingraph")
                 else float("nan")) for m in modes}
        rows.append(f"| {name} | " + " | ".join(f"{t[m]:.4f}" for m in modes) + " |")
        print(rows[-1], flush=True)
    dist.destroy_process_group()
    txt = "\n".join(rows)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
