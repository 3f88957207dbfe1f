#!/usr/bin/env python3
"""What the data-parallel code path costs the flagship step (bench.py's 2x128 online DQN at 1,835,008
envs) on ONE GPU, wire time excluded: the DP path runs over a one-rank RCCL group with world_size
forced to 2 (every all-reduce is a real RCCL launch of the whole gradient; its result is the rank's own
gradient).  Modes:

* ``single``  -- world 1: step kernel + one fused slab-reduce / Adam launch (bench.py at N = 1);
* ``sync``    -- synchronous DP (bench.py's default at N > 1): step kernel, slab reduce, RCCL all-reduce,
                 Adam, all captured in the HIP graphs;
* ``overlap`` -- ``--dp-overlap``: this step's all-reduce on RCCL's stream beside the next step's kernel
                 (one-step-delayed gradient, eager launches; chunk schedule ``auto``: static for ws since
                 profiles/r4_flagship_dp.md, the dynamic one when this ran first);
* ``single_dyn`` / ``overlap_static`` -- the same with the other chunk schedule (separates the schedule's
                 cost from the overlapped path's).

    python tools/bench_flagship_dp.py --steps 200 --warmup 20 [--modes single,sync,overlap] [--out x.md]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(mode, steps, warm, envs, group):
    from sharetrade.config import preset_config
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.envs_per_rank = envs
    world = 1 if mode.startswith("single") else 2
    cfg.engine.dp_overlap = mode.startswith("overlap")
    if mode.endswith("_dyn"):
        cfg.engine.chunk_schedule = "dynamic"
    elif mode.endswith("_static"):
        cfg.engine.chunk_schedule = "static"
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, rank=0, world_size=world, group=group if world > 1 else None)
    use_graph, _ = benchkit.prepare_steps(eng, not cfg.engine.dp_overlap, 0, 1, None, prime_reps=4)
    eng.run(warm)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    info = {"ms": ms, "graph": use_graph, "kernel": eng.step_kernel, "schedule": getattr(eng, "chunk_schedule", "")}
    del eng
    torch.cuda.empty_cache()
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--envs", type=int, default=1835008)
    ap.add_argument("--modes", default="single,sync,overlap")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
    import torch.distributed as dist

    import build as B

    B.build_all()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    group = dist.group.WORLD
    modes = a.modes.split(",")
    rows = []
    for rep in range(a.reps):
        for m in modes:
            r = _time(m, a.steps, a.warmup, a.envs, group)
            rows.append((m, rep, r))
            print(m, rep, r, flush=True)
    base = [r["ms"] for m, _, r in rows if m == "single"]
    b0 = min(base) if base else None
    lines = [f"# Flagship DP code path on one GPU ({a.envs} envs, {a.steps} timed steps, one-rank RCCL group, "
             f"world size forced to 2; `tools/bench_flagship_dp.py`)", "",
             "| mode | rep | ms / step | vs single | step kernel | schedule | HIP graphs |", "|---|---|---|---|---|---|---|"]
    for m, rep, r in rows:
        vs = f"{100 * (r['ms'] / b0 - 1):+.1f} %" if b0 else ""
        lines.append(f"| {m} | {rep + 1} | {r['ms']:.4f} | {vs} | {r['kernel']} | {r['schedule']} | {r['graph']} |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(txt)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
