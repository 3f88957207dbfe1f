#!/usr/bin/env python3
"""Config 4's fused Adam launch with and without its bias segments (which reduce the bf16 G^T rows over the batch):
what the bias reductions cost inside the memory-bound optimizer pass."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.ops import native
    from sharetrade.trainer import deep as dp

    cfg = preset_config("flagship")
    cfg.model.hidden = [1024] * 4
    cfg.agent.lr = 1e-4
    d = dp.DeepDQN(cfg, torch.device("cuda", 0), envs=16384, batch=4096, replay_capacity=1 << 20)
    for _ in range(8):
        d.act_step()
    d.update_step()
    torch.cuda.synchronize()
    full = d._adam_multi
    wonly = dp._AdamMulti()
    C.memmove(C.addressof(wonly), C.addressof(full), C.sizeof(full))
    segs = [full.seg[k] for k in range(full.nseg) if not full.seg[k].bias]
    for k, sg in enumerate(segs):
        wonly.seg[k] = sg
    wonly.nseg = len(segs)
    wonly.total = sum(sg.blocks for sg in segs)
    bonly = dp._AdamMulti()
    C.memmove(C.addressof(bonly), C.addressof(full), C.sizeof(full))
    bsegs = [full.seg[k] for k in range(full.nseg) if full.seg[k].bias]
    for k, sg in enumerate(bsegs):
        bonly.seg[k] = sg
    bonly.nseg = len(bsegs)
    bonly.total = sum(sg.blocks for sg in bsegs)
    sh = native.stream_handle()
    for name, am in (("full (bias + weight segments)", full), ("weight segments only", wonly),
                     ("bias segments only", bonly)):
        for _ in range(5):
            native.check(d.k.st_adam_multi(am, sh), "adam")
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            native.check(d.k.st_adam_multi(am, sh), "adam")
        b.record()
        torch.cuda.synchronize()
        print(f"| {name} | {am.total} blocks | {a.elapsed_time(b) / 50 * 1e3:.1f} us |", flush=True)


if __name__ == "__main__":
    main()
