#!/usr/bin/env python3
"""The reference network's geometry (203 -> 200 -> 3, fp32, QDecisionPolicyActor.scala:18-22) on the
vector engine: env-steps/s of the per-env row kernels (csrc/mlp_f32.hip) vs the batched MFMA step
(csrc/mlp_f32_mfma.hip) at several env counts, one MI355X, HIP graphs.  Preset ``intended`` (the
reference's net and AdaGrad with its quirks fixed) unless ``--preset``.

    python benchmarks/bench_f32.py [--envs 1024,16384,65536] [--paths rows,batched,batched_det] [--out x.md]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(preset, path, E, steps, warm):
    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config(preset)
    cfg.engine.dtype = "fp32"
    cfg.engine.f32_batched = "off" if path == "rows" else "on"
    # batched: fp32 atomics; batched_det: ordered split-K / column-sum partials (bit-reproducible)
    cfg.engine.f32_deterministic = "on" if path == "batched_det" else "off"
    cfg.data.source = "random_walk"
    eng = VectorEngine(cfg, device=torch.device("cuda", 0), envs=E)
    eng.capture_graph(warmup=1)
    eng.run(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(steps)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    del eng
    torch.cuda.empty_cache()
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", default="1024,16384,65536")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--preset", default="intended")
    ap.add_argument("--paths", default="rows,batched,batched_det")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import build as B

    B.build_all()
    lines = [f"# Reference geometry (203 -> 200 -> 3, fp32, preset `{a.preset}`) on the vector engine: row kernels vs "
             "batched MFMA step (`benchmarks/bench_f32.py`, 1x MI355X, HIP graphs)", "",
             "| envs | path | ms / step | env-steps/s |", "|---|---|---|---|"]
    for E in (int(x) for x in a.envs.split(",")):
        for path in a.paths.split(","):
            steps = a.steps if path != "rows" or E <= 4096 else max(5, a.steps // 10)
            ms = _time(a.preset, path, E, steps, a.warmup)
            lines.append(f"| {E} | {path} | {ms:.3f} | {E / ms * 1e3:.3e} |")
            print(lines[-1], flush=True)
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
