#!/usr/bin/env python3
"""Per-phase cycle breakdown of csrc/qstep_pipe.hip (workgroup 0, waves 0 and 4; s_memtime stamps from the
opt-in timing build csrc/ab/qstep_pipe_stamps.hip).

Usage (GPU): python tools/stamp_pipe.py [--envs 1835008] [--out profiles/x.md]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (start stamp, end stamp, name); stamp 8 = the next iteration's stamp 0
SEGMENTS = [(0, 2, "P0: features, layer 2 of Q(x) and Q(x'), dZ1, pair weight gradients"),
            (2, 3, "P0 barrier"),
            (3, 4, "P1: env step (waves 0-3) / TD (waves 4-7) beside layer 1"),
            (4, 5, "P1: TD record, env write-back, statistics, next-tile DMA issue"),
            (5, 6, "P1: partner wait, Q(x') layer-1 tail, dZ2 + dW2"),
            (6, 7, "P1: counted s_waitcnt vmcnt (previous DMA landed)"),
            (7, 8, "P1 barrier")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=7 << 18)
    ap.add_argument("--variant", default="stamps")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import build

    os.environ["SHARETRADE_AB_BUILDS"] = "1"
    build.build_all(ab=True)
    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.step_kernel = "pipe"
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, envs=a.envs)
    eng.run(5)
    torch.cuda.synchronize()
    nmy = (a.envs // 64 + eng.grid - 1) // eng.grid
    iters = 4 * nmy + 4
    st = torch.zeros(iters * 16 + 16, dtype=torch.int64, device=dev)
    eng.cfg.engine.step_variant = a.variant
    eng._qp.stamps = st.data_ptr()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    eng.step()
    ev[1].record()
    torch.cuda.synchronize()
    eng._qp.stamps = None
    eng.cfg.engine.step_variant = ""
    assert int(eng.kernel_err.sum()) == 0
    s = st.cpu().view(iters + 1, 16)[:iters].double()
    lo, hi = 8, iters - 8          # steady state only
    lines = [f"# pipe step kernel: workgroup 0 ({a.envs} envs, grid {eng.grid}, {4 * nmy} tiles; s_memtime ticks per "
             f"iteration, steady-state iterations {lo}..{hi - 1}; stamped step {ev[0].elapsed_time(ev[1]):.3f} ms)\n",
             "| segment | wave 0 (producer) | wave 4 (partner) |", "|---|---|---|"]
    for a0, a1, name in SEGMENTS:
        vals = []
        for base in (0, 8):
            b = s[lo:hi, base:base + 8]
            end = s[lo + 1:hi + 1, base] if a1 == 8 else b[:, a1]
            vals.append(float((end - b[:, a0]).mean()))
        lines.append(f"| {name} | {vals[0]:.0f} | {vals[1]:.0f} |")
    it = float((s[lo + 1:hi + 1, 0] - s[lo:hi, 0]).mean())
    lines.append(f"| iteration (stamp 0 -> stamp 0) | {it:.0f} | |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
