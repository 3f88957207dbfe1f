#!/usr/bin/env python3
"""Weight-gradient GEMM of config 4 (dW = G^T . A, bf16 in, fp32 out, K = batch 4096):
csrc/gemm_bf16.hip (split-K, atomic fp32) vs hipBLASLt (torch.mm out_dtype=fp32).
Usage (GPU): python tools/bench_dw.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import build

    build.build_all()
    from sharetrade.ops.gemm import EPI_F32, gemm_nt

    dev = torch.device("cuda", 0)
    B = 4096
    print("| out | in | K | ours us | ours TF/s | hipBLASLt us | hipBLASLt TF/s | max rel diff |")
    print("|---|---|---|---|---|---|---|---|")
    for o, i in [(1024, 256), (1024, 1024), (64, 1024), (2048, 2048)]:
        GT = torch.randn(o, B, device=dev).to(torch.bfloat16)
        AT = torch.randn(i, B, device=dev).to(torch.bfloat16)
        d1 = torch.zeros(o, i, device=dev)
        d2 = torch.zeros(o, i, device=dev)
        wt = (128, 128) if o % 128 == 0 and i % 128 == 0 else None

        def ours():
            d1.zero_()   # split-K accumulates atomically
            gemm_nt(GT, AT, d1, EPI_F32, tile=wt, splitk="auto")

        def blas():
            torch.mm(GT, AT.t(), out_dtype=torch.float32, out=d2)

        t1, t2 = timeit(ours), timeit(blas)
        ref = GT.float() @ AT.float().t()
        ours(); blas(); torch.cuda.synchronize()
        r = lambda d: float((d - ref).abs().max() / ref.abs().max())
        fl = 2.0 * o * i * B
        print(f"| {o} | {i} | {B} | {t1:.1f} | {fl / t1 / 1e6:.0f} | {t2:.1f} | {fl / t2 / 1e6:.0f} | "
              f"{r(d1):.1e} / {r(d2):.1e} |")

    # tile / split sweep (output prezeroed elsewhere in the update: zeroing not timed)
    print()
    print("| out | in | tile | split | us |")
    print("|---|---|---|---|---|")
    for o, i in [(1024, 256), (64, 1024)]:
        GT = torch.randn(o, B, device=dev).to(torch.bfloat16)
        AT = torch.randn(i, B, device=dev).to(torch.bfloat16)
        d1 = torch.zeros(o, i, device=dev)
        for t in ((128, 128), (128, 64), (64, 64)):
            if o % t[0] or i % t[1]:
                continue
            for sk in (1, 2, 4, 8, 16, 32):
                if (B // 64) % sk or B // 64 // sk < 2:
                    continue
                us = timeit(lambda: gemm_nt(GT, AT, d1, EPI_F32, tile=t, splitk=sk, prezeroed=True))
                print(f"| {o} | {i} | {t} | {sk} | {us:.1f} |")


if __name__ == "__main__":
    main()
