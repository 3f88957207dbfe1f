"""Graph-launch boundaries of the flagship engine: the same captured graph replayed back to back vs two
captured copies replayed alternately (does a replay of one graph exec wait for its previous replay
before its packets are queued?).  Bench geometry (1,835,008 envs, ws kernel); GPU-event timing.

    python tools/graph_alt_probe.py [--envs N] [--k 16] [--reps 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sharetrade.config import preset_config  # noqa: E402
from sharetrade.trainer.engine import _CAPTURE_MODE, VectorEngine  # noqa: E402


def capture(eng, k):
    s = torch.cuda.Stream(device=eng.device)
    s.wait_stream(torch.cuda.current_stream(eng.device))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
            for _ in range(k):
                eng._native_step()
    torch.cuda.current_stream(eng.device).wait_stream(s)
    return g


def timed(fn, n):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for i in range(n):
        fn(i)
    b.record()
    b.synchronize()
    return a.elapsed_time(b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=7 << 18)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    cfg = preset_config("flagship")
    eng = VectorEngine(cfg, device=torch.device("cuda", 0), envs=a.envs)
    eng.run(3)
    ga, gb = capture(eng, a.k), capture(eng, a.k)
    s1a, s1b = capture(eng, 1), capture(eng, 1)
    out = {}
    for name, fn, n, steps in (
            ("warm", lambda i: ga.replay(), 2 * a.reps, a.k),
            (f"{a.k}-step graph, same exec", lambda i: ga.replay(), a.reps, a.k),
            (f"{a.k}-step graph, two execs alternating", lambda i: (ga if i % 2 == 0 else gb).replay(), a.reps, a.k),
            (f"{a.k}-step graph, same exec (again)", lambda i: ga.replay(), a.reps, a.k),
            ("1-step graph, same exec", lambda i: s1a.replay(), a.reps * a.k, 1),
            ("1-step graph, two execs alternating", lambda i: (s1a if i % 2 == 0 else s1b).replay(), a.reps * a.k, 1)):
        ms = timed(fn, n)
        out[name] = round(ms / (n * steps), 4)
        print(f"{name}: {out[name]} ms/step", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
