#!/usr/bin/env python3
"""The act step's output layer (16,384 x 1024 -> 3 Q values, fp32 out + bias): our 64-wide padded EPI_F32 GEMM vs
hipBLASLt at the real width (torch.nn.functional.linear, bf16 in / out, and fp32 out via addmm on fp32 copies)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=100):
    for _ in range(10):
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
    E, K = 16384, 1024
    H = torch.rand(E, K, device=dev).to(torch.bfloat16)
    Wp = torch.zeros(64, K, dtype=torch.bfloat16, device=dev)
    Wp[:3] = (torch.randn(3, K, device=dev) * 0.02).to(torch.bfloat16)
    bp = torch.zeros(64, device=dev)
    bp[:3] = torch.randn(3, device=dev)
    Q = torch.empty(E, 64, device=dev)
    W3, b3 = Wp[:3].contiguous(), bp[:3].contiguous()
    b3b = b3.to(torch.bfloat16)
    t = gm.pick_tile(E, 64)
    ours = timeit(lambda: gm.gemm_nt(H, Wp, Q, gm.EPI_F32, tile=t, bias=bp))
    lib_bf = timeit(lambda: torch.nn.functional.linear(H, W3, b3b))
    ref = (H.float() @ W3.float().t() + b3)
    got = torch.nn.functional.linear(H, W3, b3b).float()
    print(f"| ours, 64-wide padded EPI_F32 (tile {t}) | {ours:.1f} us |")
    print(f"| hipBLASLt F.linear N=3 (bf16 out) | {lib_bf:.1f} us | max rel err {float((got - ref).abs().max() / ref.abs().max()):.2e} |")


if __name__ == "__main__":
    main()
