#!/usr/bin/env python3
"""Config 4's first-layer weight gradient dW0 = G0^T . X (1024 x 256, K = batch 4096, split-K fp32): tile and
K-split sweep (the production plan: 64x64 tiles, split to ~256 workgroups)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    O, I, B = 1024, 256, 4096
    A = (torch.randn(O, B, device=dev) * 0.01).to(torch.bfloat16)
    X = torch.rand(I, B, device=dev).to(torch.bfloat16)
    out = torch.zeros(O, I, device=dev)
    ref = None
    for tile in ((64, 64), (128, 64), (128, 128)):
        for sk in (1, 2, 4, 8, 16):
            if (B // 64) % sk:
                continue

            def run():
                gm.gemm_nt(A, X, out, gm.EPI_F32, tile=tile, splitk=sk)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(50):
                run()
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / 50 * 1e3
            if ref is None:
                ref = out.clone()
            err = float((out - ref).abs().max() / ref.abs().max())
            wg = (O // tile[0]) * (I // tile[1]) * sk
            print(f"| {tile} | {sk} | {wg} | {us:.1f} us | {err:.1e} |", flush=True)


if __name__ == "__main__":
    main()


def lib():
    """hipBLASLt with bf16 operands and an fp32 output (torch.mm(..., out_dtype=torch.float32)) at the same shape."""
    dev = torch.device("cuda", 0)
    O, I, B = 1024, 256, 4096
    A = (torch.randn(O, B, device=dev) * 0.01).to(torch.bfloat16)
    X = torch.rand(I, B, device=dev).to(torch.bfloat16)
    ref = A.float() @ X.float().t()

    def run():
        return torch.mm(A, X.t(), out_dtype=torch.float32)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        out = run()
    b.record()
    torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    print(f"| hipBLASLt mm, fp32 out | - | - | {a.elapsed_time(b) / 50 * 1e3:.1f} us | {err:.1e} |", flush=True)


if __name__ == "__main__" and "--lib" in sys.argv:
    lib()
