#!/usr/bin/env python3
"""TFLOP/s of the bf16 MFMA GEMM on the deep-MLP learner shapes, vs torch.matmul (hipBLASLt)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


TILES_AB = [(128, 128), (256, 128), (256, 256), (128, 128, 3), (128, 128, 4)]


def main():
    import build

    build.build_all()
    from sharetrade.ops.gemm import EPI_BF16, EPI_F32, gemm_nt, pick_tile

    shapes = [(4096, 1024, 1024), (4096, 1024, 256), (1024, 1024, 4096), (16384, 1024, 1024), (8192, 8192, 8192)]
    rows = ["| M | N | K | tile | ours TF/s (bf16 out) | ours TF/s (fp32 out) | torch.matmul TF/s |", "|---|---|---|---|---|---|---|"]
    for M, N, K in shapes:
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        o16 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        o32 = torch.empty(M, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * K
        tt = timeit(lambda: torch.matmul(A, B.t()))
        tiles = [pick_tile(M, N)] + [t for t in TILES_AB if t != pick_tile(M, N) and M % t[0] == 0 and N % t[1] == 0]
        for t in tiles:
            t16 = timeit(lambda: gemm_nt(A, B, o16, EPI_BF16, relu=True, tile=t))
            t32 = timeit(lambda: gemm_nt(A, B, o32, EPI_F32, tile=t))
            rows.append(f"| {M} | {N} | {K} | {t} | {fl / t16 / 1e12:.0f} | {fl / t32 / 1e12:.0f} | "
                        f"{fl / tt / 1e12:.0f} |")
    txt = "\n".join(rows) + "\n"
    print(txt)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write("# bf16 GEMM throughput (random operands)\n\n" + txt)


if __name__ == "__main__":
    main()
