#!/usr/bin/env python3
"""Config 4's act-step layers (16,384 rows) on our GEMM kernels (auto tile: the 256x256 ping-pong) vs the
library path (hipBLASLt through torch: addmm + fused ReLU epilogue where torch offers it).

    python tools/bench_act_gemm.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    print("| M x K -> N | ours us (tile) | torch addmm+relu us | torch _addmm_activation us | max rel diff |")
    print("|---|---|---|---|---|")
    for (M, K, N, relu) in ((16384, 256, 1024, True), (16384, 1024, 1024, True), (16384, 1024, 64, False)):
        x = (torch.randn(M, K, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g).float()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_ours = timeit(lambda: gm.gemm_nt(x, w, out, gm.EPI_BF16, bias=b, relu=relu))
        ref = out.float().clone()
        bb = b.to(torch.bfloat16)
        t_lib = timeit(lambda: torch.relu_(torch.addmm(bb, x, w.t())) if relu else torch.addmm(bb, x, w.t()))
        try:
            t_act = timeit(lambda: torch._addmm_activation(bb, x, w.t(), use_gelu=False))
            lib = torch._addmm_activation(bb, x, w.t(), use_gelu=False).float()
        except Exception as e:  # noqa: BLE001
            t_act, lib = float("nan"), torch.relu(torch.addmm(bb, x, w.t())).float()
            print("_addmm_activation:", e)
        if not relu:
            lib = torch.addmm(bb, x, w.t()).float()
        rel = float((lib - ref).abs().max() / ref.abs().max())
        tile = gm.auto_tile(M, N, gm.EPI_BF16, {})
        print(f"| {M} x {K} -> {N} | {t_ours:.1f} {tile} | {t_lib:.1f} | {t_act:.1f} | {rel:.1e} |", flush=True)


if __name__ == "__main__":
    main()
