#!/usr/bin/env python3
"""Run one GEMM configuration a few times (for rocprofv3 counter passes): --tile pp|ppp|128|hipblaslt."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile", default="pp")
    ap.add_argument("--mnk", default="8192,8192,8192")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from sharetrade.ops import gemm as gm

    M, N, K = (int(x) for x in a.mnk.split(","))
    dev = torch.device("cuda", 0)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    tile = {"pp": (256, 256, "pp"), "ppp": (256, 256, "ppp"), "128": (128, 128)}.get(a.tile)
    for _ in range(a.reps):
        if tile is None:
            torch.matmul(A, W.t())
        else:
            gm.gemm_nt(A, W, out, gm.EPI_BF16, tile=tile)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
