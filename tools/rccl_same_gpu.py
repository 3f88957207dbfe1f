#!/usr/bin/env python3
"""Two ranks on ONE GPU over RCCL (backend "nccl"): an eager all-reduce and one captured in a HIP graph.  RCCL
normally requires one device per rank; this probes whether it runs both ranks on the same card here.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \\
        tools/rccl_same_gpu.py
"""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((1 << 20,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok_eager = bool((x == world * (world + 1) / 2).all())
    y = torch.full((1 << 20,), float(rank + 1), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dist.all_reduce(y)   # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    y.fill_(float(rank + 1))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dist.all_reduce(y)
    y.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    ok_graph = bool((y == world * (world + 1) / 2).all())
    print(f"rank {rank}/{world}: eager all-reduce {'ok' if ok_eager else 'WRONG'}, "
          f"graph-captured all-reduce {'ok' if ok_graph else 'WRONG'}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
