"""Where does the w4k GEMM differ from the 128x128 kernel?  (rows / cols / K of the mismatches)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sharetrade.ops.gemm import EPI_F32, gemm_nt  # noqa: E402

torch.manual_seed(0)
for (M, N, K) in ((256, 256, 64), (256, 256, 128), (256, 256, 320), (512, 512, 1024)):
    A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    r = torch.empty(M, N, device="cuda")
    o = torch.full((M, N), float("nan"), device="cuda")
    gemm_nt(A, B, r, EPI_F32, tile=(128, 128))
    gemm_nt(A, B, o, EPI_F32, tile=(256, 256, "w4k"))
    torch.cuda.synchronize()
    bad = (o != r)
    print(M, N, K, "mismatches", int(bad.sum()), "max", float((o - r).abs().nan_to_num(1e9).max()), flush=True)
    if bad.any():
        rows = bad.any(1).nonzero().flatten()
        cols = bad.any(0).nonzero().flatten()
        print("  rows", rows[:20].tolist(), "n", rows.numel(), " cols", cols[:20].tolist(), "n", cols.numel())
        # is the difference one K-tile's contribution?
        i, j = bad.nonzero()[0].tolist()
        d = float(o[i, j] - r[i, j])
        for kt in range(K // 32):
            part = float((A[i, 32 * kt:32 * kt + 32].float() * B[j, 32 * kt:32 * kt + 32].float()).sum())
            print(f"    kt {kt}: contribution {part:.4f}  diff {d:.4f}") if abs(abs(part) - abs(d)) < 1e-2 * max(1, abs(d)) else None
