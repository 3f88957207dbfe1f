#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel-trace) into a per-kernel table.

Usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [-o profiles/x.md]
"""
import argparse
import sqlite3
import sys


def summarise(db: str):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(
        f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
        f"from kernels group by {name_col} order by sum(end-start) desc").fetchall()
    extra = {}
    for k in ("grid_size_x", "workgroup_size_x", "lds_size", "vgpr_count", "accum_vgpr_count", "sgpr_count",
              "scratch_size"):
        if k in cols:
            extra[k] = k
    info = {}
    if extra:
        q = f"select {name_col}, " + ", ".join(extra) + f" from kernels group by {name_col}"
        for r in c.execute(q):
            info[r[0]] = dict(zip(extra, r[1:]))
    total = sum(r[2] for r in rows) or 1
    return rows, info, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("-o", "--out")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows, info, total = summarise(a.db)
    lines = []
    if a.title:
        lines.append(f"# {a.title}\n")
    lines.append("| kernel | calls | total ms | avg us | min us | max us | % | grid | wg | LDS B | VGPR | AGPR | SGPR |")
    lines.append("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, n, tot, avg, mn, mx in rows:
        i = info.get(name, {})
        short = name if len(name) < 90 else name[:87] + "..."
        lines.append(f"| `{short}` | {n} | {tot/1e6:.3f} | {avg/1e3:.2f} | {mn/1e3:.2f} | {mx/1e3:.2f} | "
                     f"{100*tot/total:.1f} | {i.get('grid_size_x','')} | {i.get('workgroup_size_x','')} | "
                     f"{i.get('lds_size','')} | {i.get('vgpr_count','')} | {i.get('accum_vgpr_count','')} | "
                     f"{i.get('sgpr_count','')} |")
    text = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
