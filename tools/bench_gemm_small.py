#!/usr/bin/env python3
"""Tile choice for the config-4 update GEMMs (4096 rows): every existing tile that divides the shape,
bf16 + bias + ReLU epilogue with and without the transposed output, vs torch.matmul."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gemm import timeit  # noqa: E402


def main():
    import build

    build.build_all()
    from sharetrade.ops.gemm import EPI_BF16, EPI_RELU_GRAD, TILES, gemm_nt, pick_tile

    shapes = [(4096, 1024, 1024), (4096, 1024, 256), (4096, 64, 1024), (16384, 1024, 1024), (16384, 1024, 256)]
    rows = ["| M | N | K | tile | fwd (bias+ReLU) TF/s | fwd + C^T TF/s | relu-grad + C^T TF/s | torch TF/s |",
            "|---|---|---|---|---|---|---|---|"]
    for M, N, K in shapes:
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        o16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        oT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
        aux = torch.randn(N, M, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        fl = 2.0 * M * N * K
        tt = timeit(lambda: torch.matmul(A, B.t()))
        for t in TILES:
            if M % t[0] or N % t[1]:
                continue
            f1 = fl / timeit(lambda: gemm_nt(A, B, o16, EPI_BF16, relu=True, bias=bias, tile=t)) / 1e12
            if t == (256, 256):
                f2 = f3 = float("nan")
            else:
                f2 = fl / timeit(lambda: gemm_nt(A, B, o16, EPI_BF16, relu=True, bias=bias, outT=oT, tile=t)) / 1e12
                f3 = fl / timeit(lambda: gemm_nt(A, B, o16, EPI_RELU_GRAD, outT=oT, auxT=aux, tile=t)) / 1e12
            mark = " (pick)" if t == pick_tile(M, N) else ""
            rows.append(f"| {M} | {N} | {K} | {t}{mark} | {f1:.0f} | {f2:.0f} | {f3:.0f} | {fl / tt / 1e12:.0f} |")
            print(rows[-1], flush=True)
    txt = "\n".join(rows) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write("# GEMM tile choice on the config-4 shapes (random operands, 1x MI355X)\n\n" + txt)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
