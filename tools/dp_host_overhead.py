#!/usr/bin/env python3
"""Host cost of one overlapped-DP engine step, measured on ONE GPU.

The multi-GPU bench runs the DP step eagerly (no graph): per step two ctypes kernel launches, a
c10d all-reduce enqueue on RCCL's stream, a stream wait and one more launch.  If that host work
exceeds the ~60 us GPU step, N>1 runs become host-bound.  This tool builds a 1-rank RCCL process
group, attaches the same GradSync to a flagship engine and drives the real `_overlap_step` path
(the all-reduce over one rank is a copy-free RCCL launch), reporting:

* host enqueue time per step (50 steps issued without a sync: nothing blocks on the GPU yet);
* steady-state time per step over 400 steps, against the same engine's 1-rank eager step.

    python tools/dp_host_overhead.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import build as _b

    _b.build_all()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from sharetrade.config import preset_config
    from sharetrade.parallel.dist import DistContext, GradSync
    from sharetrade.trainer.engine import VectorEngine

    out = {}
    for mode in ("eager_1rank", "overlap_dp", "sync_dp", "sync_dp_graph16"):
        cfg = preset_config("flagship")
        cfg.engine.dp_overlap = mode == "overlap_dp"
        eng = VectorEngine(cfg, device=dev)
        if mode != "eager_1rank":
            # the DP code path over a real (1-rank) RCCL group
            eng.world_size = 2
            eng._sync = GradSync(DistContext(0, 2, 0, "nccl", dev, dist.group.WORLD), eng.layout.numel)
        for _ in range(20):
            eng._native_step()
        torch.cuda.synchronize()
        if mode == "sync_dp_graph16":
            p_ref = eng.params.clone()
            try:
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream(device=dev)
                s.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(s):
                    eng._native_step()   # warm the collective on the capture stream
                torch.cuda.current_stream(dev).wait_stream(s)
                torch.cuda.synchronize()
                with torch.cuda.graph(g):
                    for _ in range(16):
                        eng._native_step()
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                out[mode] = {"capture_error": repr(e)[:300]}
                print(mode, out[mode], flush=True)
                continue
            t0 = time.perf_counter()
            for _ in range(25):
                g.replay()
            torch.cuda.synchronize()
            out[mode] = {"us_per_step": round((time.perf_counter() - t0) / 400 * 1e6, 1),
                         "params_changed": bool(not torch.equal(p_ref, eng.params)),
                         "finite": bool(torch.isfinite(eng.params).all())}
            print(mode, out[mode], flush=True)
            continue
        t0 = time.perf_counter()
        for _ in range(50):
            eng._native_step()
        t_enq = (time.perf_counter() - t0) / 50
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(400):
            eng._native_step()
        torch.cuda.synchronize()
        t_step = (time.perf_counter() - t0) / 400
        if mode == "overlap_dp":
            eng.flush_pending()
        out[mode] = {"host_enqueue_us_per_step": round(t_enq * 1e6, 1), "us_per_step": round(t_step * 1e6, 1)}
        print(mode, out[mode], flush=True)
    print(json.dumps(out))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
