#!/usr/bin/env python3
"""The act step's first layer (16,384 x 256 -> 1024, bf16 out, bias + ReLU): our GEMM (the tile pick_tile chooses)
vs hipBLASLt's fused bias + ReLU epilogue (torch._addmm_activation), which the act step already uses for its
1024 -> 1024 layers (sharetrade/trainer/deep.py `_forward`, ``lib``)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    for E, K, N in ((16384, 256, 1024), (16384, 1024, 1024)):
        X = torch.rand(E, K, device=dev).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device=dev) * 0.1
        bb = b.to(torch.bfloat16)
        o1 = torch.empty(E, N, dtype=torch.bfloat16, device=dev)
        o2 = torch.empty_like(o1)
        t = gm.pick_tile(E, N)
        ours = timeit(lambda: gm.gemm_nt(X, W, o1, gm.EPI_BF16, tile=t, bias=b, relu=True))
        for tt in ((256, 256, "pp"), (256, 128), (128, 128, 3)):
            us = timeit(lambda: gm.gemm_nt(X, W, o1, gm.EPI_BF16, tile=tt, bias=b, relu=True))
            print(f"| {E}x{K}->{N} | ours (tile {tt}) {us:.1f} us |", flush=True)
        lib = timeit(lambda: torch._addmm_activation(bb, X, W.t(), out=o2))
        ref = torch.relu(X.float() @ W.float().t() + b)
        e1 = float((o1.float() - ref).abs().max() / ref.abs().max())
        e2 = float((o2.float() - ref).abs().max() / ref.abs().max())
        print(f"| {E}x{K}->{N} | ours (tile {t}) {ours:.1f} us (err {e1:.1e}) | hipBLASLt {lib:.1f} us (err {e2:.1e}) |",
              flush=True)


if __name__ == "__main__":
    main()
