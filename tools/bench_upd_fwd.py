#!/usr/bin/env python3
"""The config-4 update's forward layer pair (online with C^T + target, 4096 x 1024 -> 1024, bias + ReLU): our batched
128x128 launch vs the online product on our kernel and the target product through hipBLASLt's fused epilogue (same
stream, or the target on a second stream)."""
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
    return a.elapsed_time(b) / n * 1e3


def main():
    import build

    build.build_all()
    from sharetrade.ops import gemm as gm

    dev = torch.device("cuda", 0)
    M, N, K = 4096, 1024, 1024
    bf = torch.bfloat16
    X, Xn = (torch.rand(M, K, device=dev) - 0.5).to(bf), (torch.rand(M, K, device=dev) - 0.5).to(bf)
    W, Wt = ((torch.rand(N, K, device=dev) - 0.5) * 0.05).to(bf), ((torch.rand(N, K, device=dev) - 0.5) * 0.05).to(bf)
    b, bt = torch.randn(N, device=dev) * 0.1, torch.randn(N, device=dev) * 0.1
    btb = bt.to(bf)
    H, HT, Hn = torch.empty(M, N, dtype=bf, device=dev), torch.empty(N, M, dtype=bf, device=dev), torch.empty(M, N, dtype=bf, device=dev)
    t = gm.pick_tile(M, N)

    def batched():
        gm.gemm_nt_batched([(X, W, H, dict(outT=HT, bias=b, relu=True)), (Xn, Wt, Hn, dict(bias=bt, relu=True))],
                           gm.EPI_BF16, tile=t)

    def online():
        gm.gemm_nt(X, W, H, gm.EPI_BF16, tile=t, outT=HT, bias=b, relu=True)

    def target_lib():
        torch._addmm_activation(btb, Xn, Wt.t(), out=Hn)

    def split_serial():
        online()
        target_lib()

    side = torch.cuda.Stream()

    def split_streams():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        with torch.cuda.stream(side):
            target_lib()
        online()
        main.wait_stream(side)

    for name, fn in (("batched pair (production)", batched), ("online alone (ours, C^T)", online),
                     ("target alone (hipBLASLt)", target_lib), ("online + target, one stream", split_serial),
                     ("online + target, two streams", split_streams)):
        print(f"| {name} | {timeit(fn):.1f} us |", flush=True)


if __name__ == "__main__":
    main()
