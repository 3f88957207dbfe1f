"""Disassemble one csrc/*.hip file for gfx950 and summarise a kernel's instruction mix.

    python tools/isa.py csrc/qstep_ws.hip [--kernel qstep_ws_kernel] [--out /tmp/ws.s]

Prints per-kernel VGPR / AGPR / spill counts (from the assembler's metadata) and instruction counts by class
(VALU, MFMA, DS read / write, VMEM, SALU, waitcnt).  Used to check a kernel edit's register and
instruction budget on the CPU before spending a GPU run on it.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import build  # noqa: E402


def asm(src, out, defines=()):
    cmd = [build.HIPCC] + build.HIP_FLAGS + [f"-D{d}" for d in defines] + ["--cuda-device-only", "-S", src, "-o", out]
    subprocess.run(cmd, check=True)
    return open(out).read()


def classify(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "DS read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "DS write"
    if op.startswith("ds_"):
        return "DS other"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "SALU/branch"
    if op.startswith("v_"):
        return "VALU"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--out", default="/tmp/isa_out.s")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the compile (e.g. WS_MARKS=1)")
    a = ap.parse_args()
    text = asm(a.src, a.out, a.define)
    # function bodies: "<name>:" ... ".Lfunc_end"
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", text, re.M | re.S):
        name, body = m.group(1), m.group(2)
        if a.kernel and a.kernel not in name:
            continue
        cnt = collections.Counter()
        ops = collections.Counter()
        seg = collections.defaultdict(collections.Counter)   # ";@W I" marks (WS_MARKS builds)
        cur = None
        for line in body.splitlines():
            s = line.strip()
            if s.startswith(";@"):
                cur = s[2:]
                continue
            if not s or s.startswith((";", ".", "/")) or s.endswith(":"):
                continue
            op = s.split()[0]
            cnt[classify(op)] += 1
            ops[op] += 1
            if cur is not None:
                seg[cur][classify(op)] += 1
        meta = {}
        tail = text[m.end():m.end() + 6000]
        for key in ("NumVgprs", "NumAgprs", "TotalNumVgprs", "ScratchSize", "Occupancy"):
            mm = re.search(rf"; {key}: (\d+)", tail)
            if mm:
                meta[key] = int(mm.group(1))
        print(name, meta)
        print("  " + ", ".join(f"{k} {v}" for k, v in sorted(cnt.items())))
        for k in sorted(seg, key=lambda t: (t.split()[0], int(t.split()[1]))):
            print(f"  after mark {k:6s}: " + ", ".join(f"{c} {v}" for c, v in sorted(seg[k].items())))
        print("  top VALU: " + ", ".join(f"{k} {v}" for k, v in ops.most_common(60) if k.startswith("v_") and "mfma" not in k)[:600])


if __name__ == "__main__":
    main()
