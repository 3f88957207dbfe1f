#!/usr/bin/env python3
"""Scan the gfx950 ISA of the native kernels for MFMA result hazards the compiler under-pads.

Measured on MI355X (tools/ubench/mfma_raw_gen.py, profiles/r5_mfma_hazards.md): with inline asm placing
exactly N wait states between an MFMA and the consumer of its result,

* a ``v_mfma_f32_16x16x16_bf16`` that reads a ``v_mfma_f32_16x16x32_bf16`` result as its accumulator sees
  the OLD accumulator unless >= 4 wait states separate them (x32 -> x32 and x16 -> x32 chains forward at 0);
* ``v_accvgpr_read`` of an MFMA's AGPR result needs >= 7 wait states after a 16x16x32 MFMA, >= 5 after a
  16x16x16 one;
* a VALU read of an MFMA's VGPR result, a VALU write of its A / B operands (tools/ubench/mfma_war_gen.py),
  a 16x16x32 -> 16x16x32 or 16x16x16 -> 16x16x32 accumulator chain and a bf16 result read as the
  accumulator of a ``v_mfma_scale_f32_16x16x128_f8f6f4`` are safe at 0.

hipcc (ROCm 7.2) emitted the first pattern with 1 wait state in csrc/qtarget.hip -- the 16x16x16 tail
k-step of a layer-1 tile read the accumulator before the last 16x16x32 k-step had written it, dropping that
k-step (2 % error in the target Q values; tools/debug/qt_colprobe.py found the columns).  This tool lists
every MFMA -> consumer pair closer than the measured minimum in straight-line code (a pair split by a
branch or label is not followed; an MFMA between the two counts as 4 wait states, its issue cycles), per
source file.  Exit status 1 if any is found.

    python tools/mfma_hazard_scan.py [csrc/x.hip ...]
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import build  # noqa: E402

REG = re.compile(r"^([va])(\d+)$|^([va])\[(\d+):(\d+)\]$")
# (producer opcode prefix, consumer kind) -> minimum wait states, measured
NEED_SRCC_OTHER = {"v_mfma_f32_16x16x32": 4}          # x32 result -> a 16x16x16 MFMA's SrcC
SRCC_CONSUMERS = ("v_mfma_f32_16x16x16",)
NEED_ACCREAD = {"v_mfma_f32_16x16x32": 7, "v_mfma_f32_16x16x16": 5}


def regs(tok):
    m = REG.match(tok.strip())
    if not m:
        return set()
    if m.group(1):
        return {(m.group(1), int(m.group(2)))}
    return {(m.group(3), i) for i in range(int(m.group(4)), int(m.group(5)) + 1)}


def parse(line):
    parts = line.split(None, 1)
    return parts[0], ([t.strip() for t in parts[1].split(",")] if len(parts) > 1 else [])


def need(prod_op, kind):
    table = NEED_SRCC_OTHER if kind == "srcc" else NEED_ACCREAD
    for k, v in table.items():
        if prod_op.startswith(k):
            return v
    return 0


def scan(text):
    hits = []
    fn = None
    live = []   # (producer line, opcode, dst regs, wait states since issue)
    for raw in text.splitlines():
        line = raw.split(";")[0].strip()
        if not line:
            continue
        if line.endswith(":"):
            if not line.startswith("."):
                fn = line[:-1]
            live = []
            continue
        if line.startswith("."):
            continue
        op, ops = parse(line)
        if op.startswith("s_nop"):
            n = int(ops[0], 0) + 1 if ops else 1
            live = [(p, o, d, ws + n) for p, o, d, ws in live]
            continue
        # an unconditional transfer ends the straight-line path; a conditional branch does not (its
        # fall-through continues: a loop exit that reads an accumulator right after the loop's last MFMA
        # is such a path)
        if op.startswith(("s_branch", "s_setpc", "s_endpgm")):
            live = []
            continue
        if op.startswith("s_cbranch"):
            continue
        if op.startswith("v_mfma") and len(ops) >= 4:
            srcc = regs(ops[3])
            for p, o, d, ws in live:
                if op.startswith(SRCC_CONSUMERS) and srcc & d and ws < need(o, "srcc"):
                    hits.append((fn, "SrcC", ws, need(o, "srcc"), p, line))
        elif op in ("v_accvgpr_read_b32", "v_accvgpr_mov_b32") and len(ops) >= 2:   # (mov: AGPR source, unmeasured; same rule)
            src = regs(ops[1])
            for p, o, d, ws in live:
                if src & d and ws < need(o, "acc"):
                    hits.append((fn, "accvgpr_read", ws, need(o, "acc"), p, line))
        # an intervening MFMA holds the next one's issue for its own passes (>= 4 cycles)
        step = 4 if op.startswith("v_mfma") else 1
        live = [(p, o, d, ws + step) for p, o, d, ws in live]
        if op.startswith("v_mfma") and ops:
            live.append((line, op, regs(ops[0]), 0))
        live = [x for x in live if x[3] < 8]
    return hits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--defines", default="", help="comma-separated -D macros (e.g. for csrc/ab builds)")
    a = ap.parse_args()
    srcs = a.sources or sorted(glob.glob(os.path.join(ROOT, "csrc", "*.hip")))
    defs = [f"-D{d}" for d in a.defines.split(",") if d]
    total = 0
    with tempfile.TemporaryDirectory() as d:
        def compile_one(src):
            out = os.path.join(d, os.path.basename(src) + ".s")
            cmd = [build.HIPCC] + build.HIP_FLAGS + defs + ["--cuda-device-only", "-S", src, "-o", out]
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            return out

        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            outs = list(ex.map(compile_one, srcs))
        for src, out in zip(srcs, outs):
            hits = scan(open(out).read())
            total += len(hits)
            print(f"{os.path.relpath(src, ROOT)}: {len(hits)} under-padded MFMA result reads")
            for fn, kind, ws, nd, p, c in hits[:10]:
                print(f"    {fn[:50]}: {kind} at {ws} < {nd} wait states: {p}  ->  {c}")
    print(f"total: {total}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
