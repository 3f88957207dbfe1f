#!/usr/bin/env python3
"""Time the target-network pass (csrc/qtarget.hip) per launch variant at the bench batch, and check that the
variants agree bit for bit (same MFMA order per tile).

    python tools/bench_qtarget.py [--envs 1835008] [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=7 << 18)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.ops import native
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.agent.target_every = 1000
    eng = VectorEngine(cfg, device=torch.device("cuda", 0), envs=a.envs)
    eng.state.pos.copy_(torch.randint(0, eng.T - eng.H - 1, (eng.E,), dtype=torch.int32, device=eng.device))
    L, sh = native.lib(), native.stream_handle()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    ref = None
    for v, (tpw, nw) in native.QTARGET_VARIANTS.items():
        grid = max(1, min(cus, eng.E // (16 * tpw * nw)))
        eng.qt_buf.zero_()
        for _ in range(3):
            native.check(L.st_qtarget_launch_v(eng._qtp, grid, v, sh), "qtarget")
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.reps):
            native.check(L.st_qtarget_launch_v(eng._qtp, grid, v, sh), "qtarget")
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.reps
        out = eng.qt_buf.clone()
        same = "reference" if ref is None else ("bit-equal" if torch.equal(out, ref) else
                                               f"DIFFERS (max {float((out - ref).abs().max()):.3e})")
        ref = out if ref is None else ref
        gb = eng.E * 202 * 4 / 1e9
        print(f"| {v} | {tpw} | {nw} | {grid} | {ms * 1e3:.1f} | {gb / (ms / 1e3):.2f} | {same} |", flush=True)


if __name__ == "__main__":
    print("| variant | tiles / wave | waves / WG | grid | us / launch | window GB/s (TB/s x1000) | vs variant 0 |")
    print("|---|---|---|---|---|---|---|")
    main()
