#!/usr/bin/env python3
"""Forward-layer GEMM (bias + ReLU, bf16 out) at config-4 shapes: csrc/gemm_bf16.hip tiles vs
hipBLASLt through torch (``torch._addmm_activation``, its RELU_BIAS epilogue) vs plain torch.matmul.
Prints a markdown table (random operands, CUDA-event timing over 50 launches)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3   # us


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    rows = ["| M | N | K | ours (tile) us | ours TF/s | addmm_activation us | TF/s | max abs diff | matmul us |",
            "|---|---|---|---|---|---|---|---|---|"]
    for M, N, K in ((16384, 1024, 1024), (16384, 1024, 256), (4096, 1024, 1024), (8192, 1024, 1024),
                    (16384, 64, 1024)):
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        W = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16) * 0.05
        bias = torch.randn(N, device=dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        best = None
        for tile in ((128, 128), (256, 128), (256, 256), (256, 256, "pp"), (128, 64), (64, 64)):
            if M % tile[0] or N % tile[1]:
                continue
            t = timeit(lambda: gm.gemm_nt(A, W, out, gm.EPI_BF16, tile=tile, bias=bias, relu=True))
            if best is None or t < best[0]:
                best = (t, tile)
        ref = out.clone()
        gm.gemm_nt(A, W, ref, gm.EPI_BF16, tile=best[1], bias=bias, relu=True)
        bb = bias.to(torch.bfloat16)
        try:
            t2 = timeit(lambda: torch._addmm_activation(bb, A, W.t(), use_gelu=False))
            o2 = torch._addmm_activation(bb, A, W.t(), use_gelu=False)
            diff = float((o2.float() - ref.float()).abs().max())
        except Exception as e:  # noqa: BLE001
            t2, diff = float("nan"), repr(e)[:40]
        t3 = timeit(lambda: torch.matmul(A, W.t()))
        fl = 2.0 * M * N * K
        rows.append(f"| {M} | {N} | {K} | {best[0]:.1f} {best[1]} | {fl / best[0] / 1e6:.0f} | {t2:.1f} | "
                    f"{fl / t2 / 1e6:.0f} | {diff} | {t3:.1f} |")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
