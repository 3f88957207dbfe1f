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

SEGMENTS = ["P0: features (staged window -> X, X', env record)", "P0: layer 2 Q(x), layer 2 Q(x'), dZ1",
            "P0 barrier", "P1: env step + TD (waves 0-3)", "P1: stage DMA, layer 1, pair weight gradients",
            "P1: partner waits, Q(x') layer-1 tail, dZ2 + dW2", "P1: s_waitcnt vmcnt(0) (DMA + stores landed)",
            "P1 barrier"]


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
    for wv, base in ((0, 0), (4, 8)):
        pass
    for i, name in enumerate(SEGMENTS):
        vals = []
        for base in (0, 8):
            b = s[lo:hi, base:base + 8]
            if i < 7:
                d = b[:, i + 1] - b[:, i]
            else:
                d = s[lo + 1:hi + 1, base] - b[:, 7]
            vals.append(float(d.mean()))
        lines.append(f"| {name} | {vals[0]:.0f} | {vals[1]:.0f} |")
    it = float((s[lo + 1:hi + 1, 0] - s[lo:hi, 0]).mean())
    lines.append(f"| iteration (stamp 0 -> stamp 0) | {it:.0f} | |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
