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

PHASES = {32: ["P0 gather", "P1-3 fwd Q(x)", "P4 select+env", "P5-7 fwd Q(x')", "P8 TD+writeback",
               "P9-10 bwd data", "P11 weight grads"],
          64: ["P0 gather", "P1-2 hidden Q(x)", "P3 out Q(x)+select+env", "P4-5 hidden Q(x')",
               "P6 out Q(x')+TD+writeback", "P7-8 bwd data", "P9 weight grads"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--out", default="")
    ap.add_argument("--chunk", type=int, default=0, help="0 = engine default, 32 or 64")
    ap.add_argument("--waves", type=int, default=8, help="64-env-chunk kernel: 4 or 8 waves")
    ap.add_argument("--kernel", default="auto", help="engine.step_kernel: auto | wide | narrow | ws")
    ap.add_argument("--ws-dvariant", default="", help="ws: data-wave stamps build suffix ('' = stamps, gskipst)")
    ap.add_argument("--bank16", default="auto", help="ws: engine.bank16 (auto: u16 tick windows; off: fp32 windows)")
    a = ap.parse_args()
    if a.kernel == "ws":
        return ws_stamps(a)
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.ops import native
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.chunk = a.chunk
    cfg.engine.step_waves = a.waves
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, envs=a.envs)
    eng.run(3)
    torch.cuda.synchronize()
    iters = (a.envs // eng.chunk + eng.grid - 1) // eng.grid
    names = PHASES[eng.chunk]
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
        rows.append((names[ph], float(d.mean())))
        tot += float(d.mean())
    loop = float((s[1:, 0] - s[:-1, 0]).double().mean()) if iters > 1 else tot
    lines = [f"# fused step kernel phase breakdown (chunk {eng.chunk}, workgroup 0, {a.envs} envs, grid {eng.grid}, "
             f"{iters} chunks/WG; s_memtime ticks)\n", "| phase | ticks/chunk | % |", "|---|---|---|"]
    for n, v in rows:
        lines.append(f"| {n} | {v:.0f} | {100 * v / tot:.1f} |")
    lines.append(f"| chunk loop (stamp0->stamp0) | {loop:.0f} | |")
    if eng.chunk != 32:   # the P0 sub-stamps exist in the 32-env kernel only; it stamps prologue / epilogue
        x = st.cpu().view(-1, 16)[iters, 8:13].double()
        lines.append(f"| prologue (W0 fragments, W1/W2 -> LDS, first gather) | {float(x[1] - x[0]):.0f} | |")
        lines.append(f"| chunk loop, all chunks | {float(x[2] - x[1]):.0f} | |")
        lines.append(f"| step statistics + gradient slab write-out | {float(x[3] - x[2]):.0f} | |")
        lines.append(f"| exit | {float(x[4] - x[3]):.0f} | |")
        txt = "\n".join(lines) + "\n"
        print(txt)
        if a.out:
            open(a.out, "w").write(txt)
        return
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


def ws_stamps(a):
    """csrc/qstep_ws.hip: data wave 0 of workgroup 0 per 16-env tile, gradient wave 0 per ring slot (the
    stamps builds live in the opt-in A/B library, csrc/ab/)."""
    import build

    os.environ["SHARETRADE_AB_BUILDS"] = "1"
    build.build_all(ab=True)
    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.step_kernel = "ws"
    cfg.engine.bank16 = a.bank16
    dev = torch.device("cuda", 0)
    eng = VectorEngine(cfg, device=dev, envs=a.envs)
    eng.run(3)
    torch.cuda.synchronize()
    nmy = (a.envs // 64 + eng.grid - 1) // eng.grid

    def stamped(variant):
        # data-wave stamps from csrc/ab/qstep_ws_stamps.hip, gradient-wave stamps from csrc/ab/qstep_ws_gstamps.hip
        st = torch.zeros((nmy + 1) * 16 + 8 * 4 * nmy + 16, dtype=torch.int64, device=dev)
        eng.cfg.engine.step_variant = variant
        eng._qp.stamps = st.data_ptr()
        eng.step()
        torch.cuda.synchronize()
        eng._qp.stamps = None
        eng.cfg.engine.step_variant = ""
        assert int(eng.kernel_err.sum()) == 0
        return st.cpu()

    raw = stamped(a.ws_dvariant)
    graw = stamped("gstamps")
    s = raw[: nmy * 16].view(nmy, 16).double()
    names = ["features", "layer 1 of Q(x) + Q(x') window (56 + 48 MFMA) + Philox draw", "slot wait (own slot freed)",
             "X, H1 -> slot", "layer 2 of Q(x) (32 MFMA) + H2 -> slot", "output of Q(x) (4 MFMA chain)",
             "epsilon-greedy + env step", "Q(x'): layer-1 tail, layer 2, output (8 + 32 + 4 MFMA) + next prices issued",
             "TD + state write-back", "dZ2 (8 MFMA 16x16x16 + packed mask)", "dZ2, dQ -> slot, publish"]
    lines = [f"# ws step kernel: data wave 0 of workgroup 0 ({a.envs} envs, grid {eng.grid}, {nmy} tiles per data "
             f"wave; s_memtime ticks; build {a.ws_dvariant or 'stamps'}; windows {'u16 ticks' if eng.ticks is not None else 'fp32'})\n", "| phase | ticks/tile | % |", "|---|---|---|"]
    tot = 0.0
    rows = []
    for ph in range(11):
        d = float((s[:, ph + 1] - s[:, ph]).mean())
        rows.append((names[ph], d))
        tot += d
    for n, v in rows:
        lines.append(f"| {n} | {v:.0f} | {100 * v / tot:.1f} |")
    sub = float((s[:, 12] - s[:, 1]).mean())
    lines.append(f"| (of layer 1: philox + k-steps 0..5, 96 MFMA 16x16x32) | {sub:.0f} | |")
    loop = float((s[1:, 0] - s[:-1, 0]).mean()) if nmy > 1 else tot
    lines.append(f"| tile loop (stamp0 -> stamp0) | {loop:.0f} | |")
    g = graw[(nmy + 1) * 16: (nmy + 1) * 16 + 8 * 4 * nmy].view(4 * nmy, 8).double()
    g = g[g[:, 6] > 0]   # paired slots: one row per pair
    gn = ["wait for the next two full slots", "dZ1 of both slots (16 MFMA 16x16x32, W1^T read once) + "
          "own H1 tiles / first X fragments issued", "dZ1 mask", "dW0 (26 MFMA 16x16x32, K = 32 envs)",
          "dW1 (16 MFMA 16x16x32), bias sums, dW2 fragments, release", "dW2 (2 MFMA 16x16x32)"]
    lines += ["", "| gradient wave 0, per PAIR of ring slots (separate build) | ticks | % |", "|---|---|---|"]
    gt = float((g[:, 6] - g[:, 0]).mean())
    for i, n in enumerate(gn):
        d = float((g[:, i + 1] - g[:, i]).mean())
        lines.append(f"| {n} | {d:.0f} | {100 * d / gt:.1f} |")
    lines.append(f"| slot total | {gt:.0f} | |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
