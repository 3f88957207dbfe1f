#!/usr/bin/env python3
"""The config-4 update's two big launch shapes on the 128x128 kernel with BK 64 / 2 stages (today) vs BK 32
with 3 / 4 stages (tiles 10 / 11, gemm_dual kvar 1 / 2):
  fwd pair: online (C + C^T) and target forward of a 1024-wide layer, 2 x 4096 x 1024 x 1024, one launch;
  dual:     G_{l-1} = (G_l . W_l) * mask (C + C^T) beside dW_l = G_l^T . A_l (1024 x 1024 x 4096, split-K 4).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    import build

    build.build_all()
    from sharetrade.ops.gemm import EPI_BF16, EPI_F32, EPI_RELU_GRAD, gemm_dual, gemm_nt_batched

    M, H = 4096, 1024
    bf = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)   # noqa: E731
    X, Xn, W, Wt = bf(M, H), bf(M, H), bf(H, H), bf(H, H)
    b = torch.randn(H, device="cuda")
    o, oT, on = bf(M, H), bf(H, M), bf(M, H)
    G, WT, aux, GT, AT = bf(M, H), bf(H, H), bf(H, M), bf(H, M), bf(H, M)
    g1, g1T, dW = bf(M, H), bf(H, M), torch.zeros(H, H, device="cuda")
    print("| variant | fwd pair us | TF/s | dual us | TF/s |\n|---|---|---|---|---|")
    fl = 2 * 2.0 * M * H * H
    for name, tile, kvar in (("BK 64, 2 stages", (128, 128), 0), ("BK 32, 4 stages", (128, 128, "k32"), 1),
                             ("BK 32, 3 stages", (128, 128, "k32s3"), 2)):
        tf = timeit(lambda: gemm_nt_batched([(X, W, o, dict(outT=oT, bias=b, relu=True)),
                                             (Xn, Wt, on, dict(bias=b, relu=True))], EPI_BF16, tile=tile))
        td = timeit(lambda: gemm_dual((G, WT, g1, dict(outT=g1T, auxT=aux)), EPI_RELU_GRAD,
                                      (GT, AT, dW, dict(splitk=4, prezeroed=True)), EPI_F32, kvar=kvar))
        print(f"| {name} | {tf * 1e6:.1f} | {fl / tf / 1e12:.0f} | {td * 1e6:.1f} | {fl / td / 1e12:.0f} |", flush=True)


if __name__ == "__main__":
    main()
