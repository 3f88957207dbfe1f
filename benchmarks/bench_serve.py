#!/usr/bin/env python3
"""Policy-serving benchmark (1x MI355X): batched SelectionAction inference, flagship 2x128 bf16 Q-net.

Three measurements, one JSON line each:

1. ``kernel``: one ``csrc/qserve.hip`` launch per batch (features + 3 layers + argmax +
   epsilon-greedy), device-resident request rows, timed with HIP events over many launches;
   against the same math as PyTorch-ROCm library calls (bf16 ``F.linear`` x 3 on precomputed
   features, argmax) -- the "plain library GEMMs" path the fused kernel replaces.
2. ``graph``: the same launch replayed from a HIP graph (launch-overhead floor for small batches).
3. ``batcher``: many client threads each issuing blocking single-row requests through
   :class:`sharetrade.serve.DynamicBatcher` (pinned staging, one copy in / launch / copy out per
   batch): requests/s and per-request latency percentiles.

Synthetic request rows (geometric random-walk prices, random budget / shares); random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rows(B, H=201, seed=0):
    g = np.random.default_rng(seed)
    p = 50.0 * np.exp(np.cumsum(g.normal(0, 0.02, size=(B, H)), axis=1, dtype=np.float32), dtype=np.float32)
    budget = g.uniform(0, 5000, size=(B, 1)).astype(np.float32)
    shares = g.integers(0, 40, size=(B, 1)).astype(np.float32)
    return torch.from_numpy(np.concatenate([p, budget, shares], 1))


def time_launches(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us per launch


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,64,1024,16384,131072,1048576")
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=150, help="per client (batcher test)")
    ap.add_argument("--max-batch", type=int, default=4096)
    ap.add_argument("--max-delay-us", type=float, default=100.0)
    args = ap.parse_args()

    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.env import trading as tr
    from sharetrade.serve import DynamicBatcher, PolicyServer

    dev = torch.device("cuda", 0)
    cfg = preset_config("flagship")
    srv = PolicyServer(cfg, device=dev, backend="native")
    L = srv.layout
    flops_row = 2 * (224 * 128 + 128 * 128 + 128 * 16)   # padded MFMA work per request row
    w0 = L.w(srv.params_bf, 0)
    w1, b1 = L.w(srv.params_bf, 1), L.b(srv.params, 1).to(torch.bfloat16)
    w2, b2 = L.w(srv.params_bf, 2), L.b(srv.params, 2).to(torch.bfloat16)
    for B in [int(b) for b in args.batches.split(",")]:
        x203 = rows(B, seed=B).to(dev)
        x = torch.zeros(B, srv.ld, device=dev)   # the server's aligned staging stride (dwordx4 gather)
        x[:, :203] = x203
        x = x[:, :203]
        steps = torch.full((B,), 500.0, device=dev)
        acts = torch.empty(B, dtype=torch.int32, device=dev)
        iters = max(20, min(2000, 2_000_000 // B))
        us = time_launches(lambda: srv._kern.launch(x, acts, None, steps, seq=1), iters)
        us_unaligned = time_launches(lambda: srv._kern.launch(x203, acts, None, steps, seq=1), iters)
        # library path: features precomputed (not timed), then three bf16 linear layers + argmax
        feats = tr.features(x[:, :201], x[:, 201], x[:, 202], "relative", cfg.env.budget)
        xp = torch.zeros(B, 224, device=dev, dtype=torch.bfloat16)
        xp[:, :203] = feats.to(torch.bfloat16)
        xp[:, 203] = 1.0

        def lib():
            h = F.relu(F.linear(xp, w0))
            h = F.relu(F.linear(h, w1, b1))
            return F.linear(h, w2, b2)[:, :3].argmax(1)

        us_lib = time_launches(lib, iters)
        g = torch.cuda.CUDAGraph()
        srv._kern.launch(x, acts, None, steps, seq=1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            srv._kern.launch(x, acts, None, steps, seq=1)
        us_graph = time_launches(g.replay, iters)
        print(json.dumps({"bench": "kernel", "batch": B, "us_per_launch": round(us, 2),
                          "requests_per_s": round(B / us * 1e6, 1), "tflops": round(B * flops_row / us * 1e-6, 1),
                          "us_graph_replay": round(us_graph, 2), "us_rows_stride_203": round(us_unaligned, 2),
                          "us_torch_library_path": round(us_lib, 2),
                          "speedup_vs_library": round(us_lib / us, 2)}), flush=True)

    # ---------------------------------------------------------------- dynamic batcher, many clients
    X = rows(args.clients * 8, seed=99).numpy()
    lat = []
    lock = threading.Lock()
    with DynamicBatcher(srv, max_batch=args.max_batch, max_delay_us=args.max_delay_us) as bat:
        def client(c):
            mine = []
            for i in range(args.requests):
                t = time.perf_counter()
                bat.submit(X[(c * 8 + i) % len(X)], float(i)).result(timeout=60)
                mine.append(time.perf_counter() - t)
            with lock:
                lat.extend(mine)

        for w in range(2):   # warm-up round (pinned buffers, first launches)
            bat.submit(X[0], 0.0).result(timeout=60)
        ts = [threading.Thread(target=client, args=(c,)) for c in range(args.clients)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        el = time.perf_counter() - t0
        st = bat.stats()
    lat_us = np.asarray(lat) * 1e6
    print(json.dumps({"bench": "batcher", "clients": args.clients, "requests": len(lat),
                      "requests_per_s": round(len(lat) / el, 1), "latency_us_p50": round(float(np.percentile(lat_us, 50)), 1),
                      "latency_us_p99": round(float(np.percentile(lat_us, 99)), 1),
                      "mean_batch": round(st["mean_batch"], 1), "max_delay_us": args.max_delay_us}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
