#!/usr/bin/env python3
"""Config 4's update forward, first layer: online + target products 4096 x 256 -> 1024 (bias + ReLU, bf16 out, the
online one with its transposed copy) in one batched launch, per tile."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    B, K, N = 4096, 256, 1024
    X, Xn = (torch.rand(B, K, device=dev).to(torch.bfloat16) for _ in range(2))
    W, Wt = ((torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16) for _ in range(2))
    b, bt = torch.randn(N, device=dev) * 0.1, torch.randn(N, device=dev) * 0.1
    A, AT, An = (torch.empty(B, N, dtype=torch.bfloat16, device=dev), torch.empty(N, B, dtype=torch.bfloat16, device=dev),
                 torch.empty(B, N, dtype=torch.bfloat16, device=dev))
    for tile in ((128, 128), (128, 64), (64, 64), (256, 128), (128, 128, 3), (128, 128, 4)):
        def run():
            gm.gemm_nt_batched([(X, W, A, dict(outT=AT, bias=b, relu=True)), (Xn, Wt, An, dict(bias=bt, relu=True))],
                               gm.EPI_BF16, tile=tile)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(100):
            run()
        e1.record()
        torch.cuda.synchronize()
        print(f"| {tile} | {e0.elapsed_time(e1) / 100 * 1e3:.1f} us |", flush=True)


if __name__ == "__main__":
    main()
