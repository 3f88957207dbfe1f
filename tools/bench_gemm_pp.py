#!/usr/bin/env python3
"""Ping-pong 256x256 GEMM (csrc/gemm_bf16.hip tile 7/8) vs the 128x128 kernel and hipBLASLt over K:
separates the per-K-tile rate from fixed prologue/epilogue cost (time = a + b * K/64)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=30):
    for _ in range(5):
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
    tiles = [t for t in gm.TILES if len(t) == 3 and t[2] in ("pp", "ppp", "w4")] + [(128, 128)]
    print("| M | N | K | " + " | ".join(str(t) for t in tiles) + " | hipBLASLt |")
    print("|---" * (4 + len(tiles)) + "|")
    for M, N, K in ((16384, 1024, 256), (16384, 1024, 1024), (16384, 1024, 4096), (8192, 8192, 8192),
                    (4096, 4096, 4096)):
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        fl = 2.0 * M * N * K
        cells = []
        for t in tiles:
            us = timeit(lambda: gm.gemm_nt(A, W, out, gm.EPI_BF16, tile=t))
            cells.append(f"{us:.1f} us {fl / us / 1e6:.0f} TF")
        us = timeit(lambda: torch.matmul(A, W.t()))
        cells.append(f"{us:.1f} us {fl / us / 1e6:.0f} TF")
        print(f"| {M} | {N} | {K} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
