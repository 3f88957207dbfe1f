#!/usr/bin/env python3
"""BASELINE.json config 4: 4x1024 MLP Q-net, 1M-transition replay buffer in HBM, batch 4096.

One iteration = one env step of all E envs (act: gather -> 5 GEMMs -> select/env/replay
insert) + ``--updates`` learner updates (sample 4096 -> 10 forward GEMMs -> TD -> 9
backward GEMMs -> Adam), each captured in a HIP graph.  Prints one JSON line.
Single GPU (DP for this config reuses the flat-bucket GradSync of the flagship).
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
    ap.add_argument("--envs", type=int, default=16384)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--hidden", default="1024,1024,1024,1024")
    ap.add_argument("--replay", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=128, help="timed iterations (a multiple of --iters-per-graph)")
    ap.add_argument("--warmup", type=int, default=64, help="acting steps to pre-fill the replay ring")
    ap.add_argument("--updates", type=int, default=1)
    ap.add_argument("--dw-gemm", default="auto", help="weight-gradient GEMMs: auto | hip (own split-K kernels)")
    ap.add_argument("--serial", action="store_true", help="one stream (no concurrent GEMM chains in the update)")
    ap.add_argument("--unfused-adam", action="store_true", help="per-layer Adam + row-sum + counter launches")
    ap.add_argument("--no-pingpong", action="store_true", help="no 256x256 ping-pong GEMM for the act-step layers")
    ap.add_argument("--early-adam", action="store_true",
                    help="Adam waits for the act step's forward only (its env step may run beside Adam)")
    ap.add_argument("--act-before-fwd", action="store_true",
                    help="fork the act step right after the replay sample (beside the update's forward GEMMs) "
                         "instead of after the forward (beside the backward chain, the default)")
    ap.add_argument("--no-fuse-xt", action="store_true",
                    help="separate transpose launch for X^T instead of the replay gather writing it")
    ap.add_argument("--fuse-act", action="store_true",
                    help="the act step's forward layers grouped into the update's forward launches (one stream)")
    ap.add_argument("--act-inline", action="store_true",
                    help="the act step inside the iteration graph on the update's stream (no fork / join)")
    ap.add_argument("--no-dual-bwd", action="store_true",
                    help="weight gradients on a second stream beside each data-gradient GEMM (fork / join per layer)")
    ap.add_argument("--unbatched-fwd", action="store_true",
                    help="online / target forward as two GEMM chains (two streams) instead of one batched launch per layer")
    ap.add_argument("--no-head-qfwd", action="store_true",
                    help="the update's output-layer forward as a split-K GEMM launch instead of inside deep_head_kernel")
    ap.add_argument("--no-act-qhead", action="store_true",
                    help="the act step's output layer as the 64-wide padded fp32 GEMM instead of csrc/deep.hip qhead_kernel")
    ap.add_argument("--act-gemm", default="lib", choices=("own", "lib", "lib0"),
                    help="the act step's hidden 1024 -> 1024 layers through hipBLASLt's fused bias + ReLU epilogue "
                         "(lib, default: 0.408 vs 0.417 ms per iteration), also its first layer (lib0: +0.5 %%), or "
                         "every layer on our GEMMs (own); profiles/r6_config4_act_lib.md")
    ap.add_argument("--iters-per-graph", type=int, default=16,
                    help="capture k whole iterations into one HIP graph (one launch per k iterations; 4: 0.402-0.405 vs "
                         "0.405-0.409 ms per iteration at 1, profiles/r6_config4_head.md; 16: 0.381-0.383 vs 0.382-0.385 "
                         "at 4, profiles/r6_config5_kgraph.md)")
    ap.add_argument("--no-bias-part", action="store_true",
                    help="Adam reduces the bias gradients from G^T instead of the backward launches' column partials")
    ap.add_argument("--no-fuse-head", action="store_true",
                    help="TD and the output layer's backward as three launches instead of one")
    ap.add_argument("--no-overlap-act", action="store_true",
                    help="serial act step then update (default: the act step runs beside the update's GEMM chains "
                         "and the update samples the ring before this iteration's inserts; profiles/r2_config4_update_ab.md)")
    a = ap.parse_args()
    if a.no_pingpong:
        from sharetrade.ops import gemm as _gm

        _gm.PINGPONG = False
    import build

    build.build_all()
    from sharetrade.config import preset_config
    from sharetrade.trainer.deep import DeepDQN

    cfg = preset_config("flagship")
    cfg.model.hidden = [int(x) for x in a.hidden.split(",")]
    cfg.agent.lr = 1e-4
    dev = torch.device("cuda", 0)
    d = DeepDQN(cfg, dev, envs=a.envs, batch=a.batch, replay_capacity=a.replay, dw_gemm=a.dw_gemm,
                concurrent=not a.serial, fused_adam=not a.unfused_adam, overlap_act=not a.no_overlap_act,
                batched_fwd=not a.unbatched_fwd, dual_bwd=not a.no_dual_bwd, act_inline=a.act_inline,
                fuse_act=a.fuse_act, fuse_xt=not a.no_fuse_xt, act_after_fwd=not a.act_before_fwd,
                early_adam=a.early_adam, act_gemm=a.act_gemm, head_qfwd=not a.no_head_qfwd, act_qhead=not a.no_act_qhead, fuse_head=not a.no_fuse_head,
                bias_part=not a.no_bias_part)
    for _ in range(a.warmup):
        d.act_step()
    k = a.iters_per_graph if a.updates == 1 else 1
    d.capture(iters_per_graph=k)
    for _ in range(3):
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
    # time the two halves separately
    torch.cuda.synchronize()
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
    hid = cfg.model.hidden
    dims = [256] + hid + [64]
    mac = sum(dims[i] * dims[i + 1] for i in range(len(dims) - 1))
    upd_flop = 2.0 * a.batch * mac * 3 + 2.0 * a.batch * mac  # fwd x + bwd (2x) + fwd x' (target)
    s = d.stats_dict()
    out = {
        "metric": "env steps/sec + learner updates/sec, 4x1024 MLP Q-net, 1M HBM replay, batch 4096 (config 4)",
        "n_gpus": 1, "dtype": "bf16", "data": "synthetic random-walk price bank; random-init weights",
        "envs": a.envs, "batch": a.batch, "hidden": hid, "replay_capacity": a.replay,
        "updates_per_step": a.updates, "ms_per_iteration": round(dt / a.steps * 1e3, 4),
        "env_steps_per_s": round(a.envs * a.steps / dt, 1), "updates_per_s": round(a.updates * a.steps / dt, 1),
        "act_ms": round(t_act * 1e3, 4), "update_ms": round(t_upd * 1e3, 4),
        "update_tflops": round(upd_flop / t_upd / 1e12, 1), "replay_size": s["replay_size"],
        "mean_loss": s["loss_sum"] / max(1, s["updates"]) / a.batch,
        "concurrent_update": d.concurrent, "fused_adam": d.fused_adam, "overlap_act": d.overlap_act,
        "batched_fwd": d.batched_fwd, "pingpong_gemm": not a.no_pingpong, "dual_bwd": d.dual_bwd, "act_inline": d.act_inline, "fuse_act": d.fuse_act,
        "act_gemm": d.act_gemm, "head_qfwd": d.head_qfwd, "act_qhead": d.act_qhead, "fuse_head": d.fuse_head, "bias_part": d._bpart[0] is not None, "iters_per_graph": k,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
