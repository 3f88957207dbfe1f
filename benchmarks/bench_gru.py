#!/usr/bin/env python3
"""BASELINE.json config 5: GRU(256) recurrent Q-net on minute-bar sequences, fp8 MFMA path.

One iteration = one actor launch (all E envs advance S minute bars through the MX-fp8
GRU actor kernel, writing one replay segment each) + ``--updates`` learner updates
(B sampled segments, S+1-step unroll of online and target nets, BPTT, Adam, fp8 repack),
each captured in a HIP graph.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--seq", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--bars", type=int, default=4096)
    ap.add_argument("--replay", type=int, default=1 << 17)
    ap.add_argument("--steps", type=int, default=128, help="timed iterations (a multiple of --iters-per-graph)")
    ap.add_argument("--warmup", type=int, default=4, help="actor launches to pre-fill the replay")
    ap.add_argument("--updates", type=int, default=1)
    ap.add_argument("--grid", type=int, default=0,
                    help="actor workgroups (one per CU): 0 = auto (RecurrentDQN._auto_grid)")
    ap.add_argument("--actor-kernel", default="auto", choices=["auto", "single", "pair"],
                    help="single- or two-chunk actor kernel (auto: two-chunk when seq <= 32)")
    ap.add_argument("--iters-per-graph", type=int, default=16,
                    help="capture k (even) whole iterations into one HIP graph (one launch per k iterations; 4: "
                         "0.583-0.584 vs 0.589-0.591 ms per iteration at 1 over 200 steps; 16: 0.578 vs 0.583-0.584 at "
                         "4; profiles/r6_config5_kgraph.md)")
    ap.add_argument("--no-overlap-act", action="store_true",
                    help="serial actor launch then update (default: the actor runs beside the update after its "
                         "segments are sampled; profiles/r2_config5_overlap.md)")
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.trainer.recurrent import RecurrentDQN

    cfg = preset_config("recurrent")
    dev = torch.device("cuda", 0)
    d = RecurrentDQN(cfg, dev, envs=a.envs, seq=a.seq, batch=a.batch, bars=a.bars, replay_segments=a.replay,
                     actor_grid=a.grid, overlap_act=not a.no_overlap_act, actor_kernel=a.actor_kernel)
    a.grid = d.grid
    for _ in range(a.warmup):
        d.act()
    k = a.iters_per_graph if a.updates == 1 and not a.no_overlap_act else 1
    d.capture(iters_per_graph=k)
    for _ in range(2):
        d.iteration(a.updates)
    if k > 1:
        d.iterations(2 * k)   # the multi-iteration graph's first replays upload it to the device
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if k > 1:
        d.iterations(a.steps)
    else:
        for _ in range(a.steps):
            d.iteration(a.updates)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    for _ in range(a.steps):
        d._g_act.replay()
    torch.cuda.synchronize()
    t_act = (time.perf_counter() - t1) / a.steps
    t2 = time.perf_counter()
    for _ in range(a.steps):
        d._g_upd.replay()
    torch.cuda.synchronize()
    t_upd = (time.perf_counter() - t2) / a.steps
    H, G = 256, 768
    act_flop = 2.0 * a.envs * a.seq * (G * H + G * 32 + 3 * H)           # h part (MX-fp8) + x part + Q head
    upd_flop = 2.0 * a.batch * (a.seq + 1) * (G * H + G * 64) * 2 + 2.0 * a.batch * a.seq * G * H * 2 \
        + 2.0 * a.batch * a.seq * G * (H + 64)                           # fwd x2, bwd dh, weight grads
    s = d.stats_dict()
    out = {
        "metric": "env steps/sec + learner updates/sec, GRU(256) recurrent Q-net on minute bars, fp8 MFMA (config 5)",
        "n_gpus": 1, "dtype": "mxfp8 actor (e4m3 + E8M0 block scales), bf16 learner",
        "data": "synthetic minute bars (AR(1)+GARCH, U-shaped intraday); random-init weights",
        "envs": a.envs, "seq": a.seq, "batch_segments": a.batch, "bars": a.bars, "replay_segments": a.replay,
        "updates_per_iteration": a.updates, "ms_per_iteration": round(dt / a.steps * 1e3, 4),
        "env_steps_per_s": round(a.envs * a.seq * a.steps / dt, 1),
        "updates_per_s": round(a.updates * a.steps / dt, 2),
        "act_ms": round(t_act * 1e3, 4), "actor_env_steps_per_s": round(a.envs * a.seq / t_act, 1),
        "actor_tflops": round(act_flop / t_act / 1e12, 1),
        "update_ms": round(t_upd * 1e3, 4), "update_tflops": round(upd_flop / t_upd / 1e12, 1),
        "episodes": s["episodes"], "episode_return_mean": s["episode_return_mean"],
        "reward_per_step": s["reward_per_step"], "loss": s["loss"], "overlap_act": d.overlap_act, "iters_per_graph": k,
        "actor_grid": a.grid, "actor_kernel": d.actor_kernel,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
