#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output (per-kernel counter sums) into markdown."""
import argparse
import csv
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("-o", "--out")
    ap.add_argument("--title", default="")
    ap.add_argument("--kernels", default="qstep,reduce_optim,f32_")
    a = ap.parse_args()
    keep = a.kernels.split(",")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(a.csv)):
        k = r["Kernel_Name"]
        if not any(s in k for s in keep):
            continue
        short = k.split("(")[0].replace("void ", "")
        tot[short][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[short].add(r["Dispatch_Id"])
    lines = [f"# {a.title}\n"] if a.title else []
    for k, c in tot.items():
        n = len(disp[k])
        lines.append(f"## `{k}` ({n} dispatches; per-dispatch means)\n")
        lines.append("| counter | value |")
        lines.append("|---|---|")
        for name in sorted(c):
            lines.append(f"| {name} | {c[name] / n:,.0f} |")
        d = {x: c[x] / n for x in c}
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if x in d:
                    lines.append(f"| {x} / SQ_WAVE_CYCLES | {d[x] / d['SQ_WAVE_CYCLES']:.3f} |")
        if "SQ_LDS_BANK_CONFLICT" in d and d.get("SQ_LDS_IDX_ACTIVE"):
            lines.append(f"| LDS bank-conflict cycles / LDS active cycles | "
                         f"{d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']:.3f} |")
        lines.append("")
    txt = "\n".join(lines) + "\n"
    if a.out:
        open(a.out, "w").write(txt)
    sys.stdout.write(txt)


if __name__ == "__main__":
    main()
