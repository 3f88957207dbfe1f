#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fused step kernel (workgroup 0, s_memtime stamps).

Usage (GPU): python tools/stamp_qstep.py [--envs 65536] [--out profiles/x.md]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["P0 gather", "P1-3 fwd Q(x)", "P4 select+env", "P5-7 fwd Q(x')", "P8 TD+writeback",
          "P9-10 bwd data", "P11 weight grads"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.ops import native
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, envs=a.envs)
    eng.run(3)
    torch.cuda.synchronize()
    iters = (a.envs // 32 + eng.grid - 1) // eng.grid
    st = torch.zeros(iters * 16 + 16, dtype=torch.int64, device=dev)
    eng._qp.stamps = st.data_ptr()
    eng.step()
    torch.cuda.synchronize()
    eng._qp.stamps = None
    s = st.cpu().view(-1, 16)[:iters]
    rows = []
    tot = 0
    for ph in range(7):
        d = (s[:, ph + 1] - s[:, ph]).double()
        rows.append((PHASES[ph], float(d.mean())))
        tot += float(d.mean())
    loop = float((s[1:, 0] - s[:-1, 0]).double().mean()) if iters > 1 else tot
    lines = [f"# fused step kernel phase breakdown (workgroup 0, {a.envs} envs, grid {eng.grid}, "
             f"{iters} chunks/WG; s_memtime ticks)\n", "| phase | ticks/chunk | % |", "|---|---|---|"]
    for n, v in rows:
        lines.append(f"| {n} | {v:.0f} | {100 * v / tot:.1f} |")
    lines.append(f"| chunk loop (stamp0->stamp0) | {loop:.0f} | |")
    wait = float((s[:, 8] - s[:, 0]).double().mean())
    lines.append(f"| of P0: waiting for prefetched loads/stores (debug waitcnt) | {wait:.0f} | |")
    rows_t = float((s[:, 9] - s[:, 8]).double().mean())
    pre_t = float((s[:, 10] - s[:, 9]).double().mean())
    bar_t = float((s[:, 1] - s[:, 10]).double().mean())
    lines.append(f"| of P0: feature rows -> LDS | {rows_t:.0f} | |")
    lines.append(f"| of P0: issue next chunk's loads | {pre_t:.0f} | |")
    lines.append(f"| of P0: barrier | {bar_t:.0f} | |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
