#!/usr/bin/env python3
"""Timeline of the last N kernels of a rocprofv3 kernel-trace database (rocpd): start offset, duration,
gap to the previous kernel's end on ANY queue, queue id, grid / workgroup sizes and the kernel name.
Concurrency shows as overlapping [start, end) on different queues.

Usage: python tools/prof_timeline.py gpurun_out/deepprof/run_results.db --last 40 [-o profiles/x.md]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name).replace("void ", "")
    return n if len(n) <= 70 else n[:67] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--title", default="")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select start, end, name, queue_id, grid_x, workgroup_x from kernels order by start").fetchall()
    rows = rows[-a.last:]
    t0 = rows[0][0]
    lines = [f"# {a.title}", ""] if a.title else []
    lines += ["| start us | dur us | gap us | queue | grid | wg | kernel |", "|---|---|---|---|---|---|---|"]
    last_end = None
    for s, e, n, q, gx, wx in rows:
        gap = "" if last_end is None else f"{(s - last_end) / 1e3:.1f}"
        lines.append(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.1f} | {gap} | {q} | {gx // max(wx, 1)} | {wx} | "
                     f"`{short(n)}` |")
        last_end = e if last_end is None else max(last_end, e)
    span = (max(r[1] for r in rows) - t0) / 1e3
    busy = sum(r[1] - r[0] for r in rows) / 1e3
    lines += ["", f"{len(rows)} kernels over {span:.1f} us; summed kernel time {busy:.1f} us "
                  f"(> span where kernels overlap)."]
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
