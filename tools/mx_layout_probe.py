#!/usr/bin/env python3
"""Empirically map the operand layout of v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950).

For every A-fragment position (lane la, byte ja) a single 1.0 is placed there and B is
filled with values that encode B's (lane group, byte) -> the non-zero D row gives A's row,
the D values give which B (lane group, byte) it was paired with.  Then the scale lane
that multiplies A (la, ja) is found by doubling one lane's scale at a time.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sharetrade.ops.gru import mx_probe  # noqa: E402


def f8(x):
    return x.to(torch.float8_e4m3fn).view(torch.uint8).cuda()


def main():
    dev = "cuda"
    ones = torch.full((64,), 127, dtype=torch.int32, device=dev)
    lane = torch.arange(64)[:, None].expand(64, 32)
    byte = torch.arange(32)[None, :].expand(64, 32)
    Bg = f8(((lane >> 4) + 1).float())
    Bj0 = f8((byte % 8 + 1).float())
    Bj1 = f8((byte // 8 + 1).float())
    out = {}
    for la in range(64):
        for ja in range(32):
            A = torch.zeros(64, 32)
            A[la, ja] = 1.0
            A8 = f8(A)
            D1 = mx_probe(A8, Bg, ones, ones).cpu()
            D2 = mx_probe(A8, Bj0, ones, ones).cpu()
            D3 = mx_probe(A8, Bj1, ones, ones).cpu()
            rows = torch.nonzero(D1.abs().sum(1)).flatten().tolist()
            if len(rows) != 1:
                out[f"{la},{ja}"] = {"rows": rows}
                continue
            i0 = rows[0]
            gb = (D1[i0] - 1).round().int().tolist()
            jb = ((D3[i0] - 1) * 8 + (D2[i0] - 1)).round().int().tolist()
            out[f"{la},{ja}"] = {"row": i0, "b_group": sorted(set(gb)), "b_byte": sorted(set(jb))}
    # scale: which A-scale lane multiplies A(la, ja)?
    scl = {}
    Ball = f8(torch.ones(64, 32))
    for la, ja in ((0, 0), (0, 31), (17, 5), (33, 16), (63, 31), (5, 20)):
        A = torch.zeros(64, 32)
        A[la, ja] = 1.0
        A8 = f8(A)
        base = mx_probe(A8, Ball, ones, ones).cpu().abs().sum()
        hits = []
        for ls in range(64):
            s = ones.clone()
            s[ls] = 128
            v = mx_probe(A8, Ball, s, ones).cpu().abs().sum()
            if abs(float(v) - 2 * float(base)) < 1e-3:
                hits.append(ls)
        scl[f"{la},{ja}"] = hits
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/mx_layout.json", "w") as f:
        json.dump({"a": out, "scale": scl}, f)
    # compact summary: hypothesis k = 32*(la>>4) + ja paired with same (group, byte) in B
    bad = [k for k, v in out.items() if not ("row" in v and v["row"] == int(k.split(",")[0]) % 16
                                             and v["b_group"] == [int(k.split(",")[0]) >> 4]
                                             and v["b_byte"] == [int(k.split(",")[1])])]
    print("positions violating the simple hypothesis:", len(bad))
    for k in bad[:40]:
        print(k, out[k])
    print("scale lanes:", scl)


if __name__ == "__main__":
    main()
