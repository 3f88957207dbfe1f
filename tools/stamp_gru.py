#!/usr/bin/env python3
"""Phase breakdown of the GRU actor kernel (csrc/gru.hip gru_act_kernel) from s_memtime stamps
of workgroup 0 / chunk 0, waves 0 (env wave) and 1.  Prints a markdown table."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--seq", type=int, default=16)
    ap.add_argument("--out", default=None)
    ap.add_argument("--kernel", default="single", choices=["single", "pair"])
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.trainer.recurrent import RecurrentDQN

    d = RecurrentDQN(preset_config("recurrent"), torch.device("cuda", 0), envs=a.envs, seq=a.seq, batch=1024,
                     bars=4096, replay_segments=1 << 17, actor_kernel=a.kernel)
    st = torch.zeros(a.seq * 2 * 8 + a.seq * 8, dtype=torch.int64, device="cuda")
    for _ in range(3):
        d.act()
    for args in d._acts:
        args.stamps = st.data_ptr()
    d.act()
    torch.cuda.synchronize()
    for args in d._acts:
        args.stamps = None
    allst = st.cpu().numpy().astype(np.int64)
    s = allst[:a.seq * 16].reshape(a.seq, 2, 8)
    arr = allst[a.seq * 16:].reshape(a.seq, 8)   # single kernel: every wave's arrival at barrier 1
    if a.kernel == "pair":
        names = ["env A (wave 0) / -", "MFMA B", "barrier + reset A", "env B (wave 0) / -", "MFMA A (next step)",
                 "barrier + reset B"]
        lines = ["# two-chunk GRU actor interval breakdown (WG 0, first pair; s_memtime ticks, mean over steps "
                 "1..S-2; one row-set = one step of BOTH chunks)", "", "| interval | wave 0 | wave 4 (same SIMD) |",
                 "|---|---|---|"]
        for i, n in enumerate(names):
            d0 = np.mean(s[1:-1, 0, i + 1] - s[1:-1, 0, i])
            d1 = np.mean(s[1:-1, 1, i + 1] - s[1:-1, 1, i])
            lines.append(f"| {n} | {d0:.0f} | {d1:.0f} |")
        step = np.mean(s[2:-1, 0, 0] - s[1:-2, 0, 0])
        lines.append(f"| two chunk-steps (stamp0 -> stamp0) | {step:.0f} | |")
        lines.append(f"| per chunk-step | {step / 2:.0f} | |")
        txt = "\n".join(lines)
        print(txt)
        if a.out:
            open(a.out, "w").write(txt + "\n")
        return
    names = ["MFMA tile 0 (x + h parts)", "tile 1 MFMA + GRU update + Q partials", "quantize h -> fp8 LDS",
             "barrier 1", "env phase (wave 0) / idle", "barrier 2 + h reset", ]
    lines = ["# GRU actor step phase breakdown (WG 0, chunk 0; s_memtime ticks, mean over steps 1..S-1)", "",
             "| phase | wave 0 | wave 1 |", "|---|---|---|"]
    for i, n in enumerate(names):
        d0 = np.mean(s[1:, 0, i + 1] - s[1:, 0, i])
        d1 = np.mean(s[1:, 1, i + 1] - s[1:, 1, i])
        lines.append(f"| {n} | {d0:.0f} | {d1:.0f} |")
    step = np.mean(s[2:, 0, 0] - s[1:-1, 0, 0])
    lines.append(f"| step (stamp0 -> stamp0) | {step:.0f} | |")
    rel = arr[1:] - s[1:, 0, 0][:, None]
    lines += ["", "arrival at barrier 1 after the step start, per wave (mean over steps 1..S-1): " +
              ", ".join(f"w{w} {np.mean(rel[:, w]):.0f}" for w in range(8))]
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
