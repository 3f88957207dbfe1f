#!/usr/bin/env python3
"""Flagship benchmark: env steps/sec (whole node) + episode return, 2x128 MLP Q-net.

BASELINE.json config 2/3: a 2-layer 128-hidden MLP Q-network in bf16, online
Q-learning (select -> env step -> TD update -> Adam) over ``--envs`` vectorised
Buy/Sell/Hold trading envs per GPU on synthetic random-walk price series
(6,047 days each, like the reference's MSFT file) with random-init weights;
one process per GPU, gradients all-reduced every step with RCCL.  Default
1,835,008 envs per GPU (weak scaling: per-GPU work fixed as N grows); the env
state, the per-env price banks and their aligned replicas stay resident in HBM
(~225 of the 309 GB per GPU).

Single GPU:   python bench.py --steps 200 --warmup 20
N GPUs:       python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                  --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Every timed step is a full learner step (all envs act, every env's TD error
is back-propagated, the optimizer updates all parameters); nothing is skipped.
After the timed window (untimed) every env plays one complete 5,846-step episode
with the policy being learned and one with a uniformly random policy: the
"episode return" half of the metric (final portfolio - budget, mean / std over
all envs of all ranks).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env steps/sec (whole node) + episode return, 2x128 MLP Q-net at 1/2/4/8 MI355X"
REFERENCE_FLOOR = 58.0  # derived minimum throughput of the reference app; not a published number


STABLE_RAMP = 500.0   # exploit ramp of the stabilised learner over the bench's ~281 training steps (r6 sweep)


def learner_knobs_on(cfg) -> bool:
    a = cfg.agent
    return bool(a.target_every or a.double_dqn or a.reward_scale != 1.0 or a.ramp_mode != "position")


def stable_learner_eval(args, dev, rank, world, group, train_steps):
    """Train preset flagship_stable (target net refreshed every 1,000 steps + Double DQN + reward scale 100 + gamma
    0.99, exploit ramp STABLE_RAMP) on the same banks for ``train_steps`` steps, then one greedy frozen episode per
    env: the learner that beats a random policy's median on this bank (profiles/r6_learner_breakdown.md)."""
    from sharetrade.config import preset_config
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship_stable")
    cfg.engine.envs_per_rank = args.envs
    cfg.agent.ramp = STABLE_RAMP
    eng = VectorEngine(cfg, device=dev, rank=rank, world_size=world, group=group)
    eng.sync_params_from(0)
    benchkit.prepare_steps(eng, not args.no_graph, rank, world, group, prime_reps=8 if world > 1 else 16,
                           fixed_prime=True)
    if train_steps > eng.step_count:
        eng.run(train_steps - eng.step_count)
    eng.synchronize()
    g = benchkit.greedy_episode_returns(eng, world, group)
    res = {"preset": "flagship_stable", "ramp": STABLE_RAMP, "train_steps": eng.step_count,
           "greedy_mean": round(g["mean"], 4), "greedy_std": round(g["std"], 4), "greedy_median": round(g["median"], 4)}
    del eng
    torch.cuda.empty_cache()
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--envs", type=int, default=int(os.environ.get("SHARETRADE_BENCH_ENVS", 7 << 18)),
                    help="vectorised envs per GPU (default 1,835,008 = 112 64-env chunks per CU: ~225 GB of the "
                         "309 GB HBM per GPU, mostly the per-env price banks; fixed per-step costs amortised, "
                         "profiles/r2_env_sweep.md)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) | gloo (rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on cuda:0 (multi-rank rehearsal on a 1-GPU box, with --dist-backend gloo)")
    ap.add_argument("--trace", default="", help="write a torch.profiler chrome trace here")
    ap.add_argument("--step-kernel", default="auto",
                    help="fused step kernel: auto | ws (flagship) | wide (64-env chunks) | narrow")
    ap.add_argument("--step-waves", type=int, default=8, help="64-env-chunk kernel: waves per workgroup (4 or 8)")
    ap.add_argument("--step-variant", default="", help="timing / debug build of the ws kernel (csrc/ab/qstep_ws_<v>.hip; needs SHARETRADE_AB_BUILDS=1)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="envs per chunk of the fused step kernel: 0 = auto (64 when envs %% 64 == 0), 32, 64")
    ap.add_argument("--dp-overlap", action="store_true",
                    help="N>1: all-reduce of step t on RCCL's stream under step t+1's kernel (one-step delayed "
                         "gradient, eager launches) instead of sync DP captured in HIP graphs (the default: "
                         "measured faster, tools/dp_host_overhead.py)")
    ap.add_argument("--sync-dp", action="store_true", help="(default) strict synchronous DP")
    ap.add_argument("--chunk-schedule", default="auto",
                    help="step-kernel chunk schedule: auto (static; dynamic for the wide kernel under overlapped DP) | static | dynamic")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps per HIP-graph replay in the timed loop (0 = engine.graph_steps)")
    ap.add_argument("--pg-timeout", type=float, default=300.0,
                    help="N>1: collective timeout (s); with TORCH_NCCL_ASYNC_ERROR_HANDLING=1 a dead peer fails "
                         "the job instead of hanging it")
    ap.add_argument("--no-episode", action="store_true",
                    help="skip the untimed full-episode returns after the timed window (greedy learned policy, "
                         "greedy random-init policy, buy-and-hold, online learned episode, random policy)")
    ap.add_argument("--target-every", type=int, default=0,
                    help="learning knob: target network refreshed every N steps (csrc/qtarget.hip pass per step)")
    ap.add_argument("--double-dqn", action="store_true", help="learning knob: Double DQN (needs --target-every)")
    ap.add_argument("--reward-scale", type=float, default=1.0, help="learning knob: reward multiplier in the TD target")
    ap.add_argument("--ramp-mode", default="position", help="learning knob: exploit ramp over 'position' | 'global'")
    ap.add_argument("--no-stable-eval", action="store_true",
                    help="skip the untimed evaluation of the stabilised learner (preset flagship_stable: target net + "
                         "Double DQN, trained for the same number of steps on the same banks)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # native build BEFORE any process group exists (build.build_all serialises concurrent builders
    # with a file lock): no rank waits in a collective while another compiles
    import build as _build  # in-tree native build (no-op when up to date)

    _build.build_all()
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    local = 0 if args.same_device else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    group = None
    if world > 1:
        import datetime

        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # the DP step is captured in HIP graphs with its RCCL all-reduce: no user-buffer registration
        # of captured collectives (it goes through IPC handles; the pool's driver is dmabuf-only)
        os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
        # a dead or stuck peer fails the job within the collective timeout instead of hanging it
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = {"device_id": dev} if args.dist_backend == "nccl" else {}
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.pg_timeout), **kw)
        group = dist.group.WORLD
        world = dist.get_world_size(group)   # as the communicator sees it

    from sharetrade.config import preset_config
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.envs_per_rank = args.envs
    cfg.engine.dp_overlap = bool(args.dp_overlap) and world > 1
    cfg.engine.chunk = args.chunk
    cfg.engine.step_waves = args.step_waves
    cfg.engine.step_kernel = args.step_kernel
    cfg.engine.step_variant = args.step_variant
    cfg.engine.chunk_schedule = args.chunk_schedule
    if args.graph_steps:
        cfg.engine.graph_steps = args.graph_steps
    cfg.agent.target_every, cfg.agent.double_dqn = args.target_every, bool(args.double_dqn)
    cfg.agent.reward_scale, cfg.agent.ramp_mode = args.reward_scale, args.ramp_mode
    eng = VectorEngine(cfg, device=dev, rank=rank, world_size=world, group=group)
    eng.sync_params_from(0)
    init_params = None if args.no_episode else eng.params.detach().clone()   # the frozen-init baseline

    # load the (lazily loaded) torch kernels of the start-of-window portfolio snapshot before the graphs
    # are primed: loading them between the warm-up and the timed window idled the GPU for >= 10 ms,
    # and the clock then needs ~40 steps to settle (tools/dvfs_probe.py, profiles/r2_dvfs_probe.md)
    eng.current_portfolios().double().clone()
    torch.cuda.synchronize()
    # capture -> vote (all ranks agree on graphs vs eager) -> prime with the same step counts on every
    # rank (each step holds the DP all-reduce); untimed, reported as "graph_prime_steps"
    # a fixed 16 multi-step replays (256 steps; the clock settles within ~13 on every box measured): the
    # policy evaluated after the window has trained the same number of steps on every run
    use_graph, _ = benchkit.prepare_steps(eng, not args.no_graph and not cfg.engine.dp_overlap, rank, world,
                                          group, prime_reps=8 if world > 1 else 16, fixed_prime=True)
    prime_steps = eng.step_count
    eng.run(args.warmup)
    eng.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    # start-of-window portfolio (window_return_mean: the portfolio change over the timed window)
    pf0 = eng.current_portfolios().double().clone()
    prof = None
    if args.trace:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    eng.run(args.steps)   # whole multi-step graph replays (engine.graph_steps) + single steps
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    if prof is not None:
        prof.__exit__(None, None, None)
        prof.export_chrome_trace(args.trace)
    eng.check_kernel_err()   # (untimed) a ws ring-protocol abort in the window would make its gradients invalid
    trained_steps = eng.step_count   # prime + warm-up + timed: what the evaluated policy has learned from
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    pf1 = eng.current_portfolios().double()
    # per-env return over the window (episode resets inside the window are rare: 5,846-step episodes)
    ret = torch.stack([(pf1 - pf0).sum(), torch.tensor(float(eng.E), dtype=torch.float64, device=dev)])
    stats = eng.stat_acc.clone() if eng.backend == "native" else eng.stats.to(dev)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(ret)
        dist.all_reduce(stats)
    el = float(elapsed[0])
    allreduce_ms = None
    if world > 1 and eng._sync is not None:
        # latency of the gradient all-reduce (same size, same group), measured AFTER the timed window
        scratch = torch.zeros_like(eng.params)
        eng._sync.enable_timing()
        for _ in range(20):
            eng._sync.all_reduce(scratch)
        ms = eng._sync.pop_timing_ms()
        eng._sync.enable_timing(False)
        t = torch.tensor([ms if ms is not None else 0.0], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        allreduce_ms = round(float(t[0]), 4)
    total_steps = eng.E * world * args.steps
    value = total_steps / el
    n_trans = eng.E * world * eng.step_count   # every step taken (prime + warmup + timed)
    st = stats.cpu().tolist()
    episodes = None
    episode_error = None
    if not args.no_episode:
        # untimed, after the timed window, every env plays complete episodes over its series
        # (T - H = 5,846 steps each) on the same banks:
        #  * greedy: the parameters learned so far, frozen, exploit-only (the policy itself);
        #  * init_greedy: the same with the random-init parameters (what learning has to improve on);
        #  * buy_hold: Buy at every step (budget into shares at the start, then held);
        #  * learned: the online epsilon-greedy episode with learning on (the training regime);
        #  * greedy_trained: greedy + frozen again, with the parameters at the end of that online episode;
        #  * random: uniformly random actions.
        try:
            greedy = benchkit.greedy_episode_returns(eng, world, group)
            init_greedy = benchkit.greedy_episode_returns(eng, world, group, params=init_params)
            buy_hold = benchkit.buy_and_hold_returns(eng, world, group)
            learned = benchkit.full_episode_returns(eng, world, group)
            # the parameters after that whole online episode (~6,000 Adam steps in all), greedy and frozen
            greedy_trained = benchkit.greedy_episode_returns(eng, world, group)
            rnd = benchkit.full_episode_returns(eng, world, group, random_policy=True)
            episodes = {"learned": learned, "random": rnd, "greedy": greedy, "init_greedy": init_greedy,
                        "buy_hold": buy_hold, "greedy_trained": greedy_trained}
        except Exception as e:  # noqa: BLE001 -- the timed measurement above stands; report what failed
            if world > 1:
                raise          # (a rank that stops mid-collective would hang its peers: fail the job)
            episode_error = f"{type(e).__name__}: {str(e).splitlines()[0] if str(e) else ''}"
            print(f"bench.py: episode evaluation failed: {episode_error}", file=sys.stderr)
    # per-rank device-memory peak of this process's allocations (torch caching allocator: every engine buffer),
    # gathered so a rank-0-only allocation that grows with the world size would show
    peak = torch.tensor([torch.cuda.max_memory_allocated(dev) / 1e9], dtype=torch.float64, device=dev)
    peaks = [peak]
    if world > 1:
        peaks = [torch.zeros_like(peak) for _ in range(world)]
        torch.distributed.all_gather(peaks, peak)
    # the stabilised learner (untimed, after everything above): the plain learner's greedy policy chases momentum on
    # this bank and loses to a uniformly random one on the median (profiles/r6_learner_breakdown.md); Double DQN
    # with a target network does not.  Same banks, same number of training steps, then the same greedy episode.
    stable = None
    if episodes is not None and not args.no_stable_eval and not learner_knobs_on(cfg):
        try:
            stable = stable_learner_eval(args, dev, rank, world, group, trained_steps)
        except Exception as e:  # noqa: BLE001 -- the timed measurement above stands
            if world > 1:
                raise
            stable = {"error": f"{type(e).__name__}: {str(e).splitlines()[0] if str(e) else ''}"}
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (per-env geometric random-walk price series, 6047 days; random-init weights)",
            "config": {
                "model": "2x128 MLP Q-net (203->128->128->3), online DQN, Adam",
                "global_batch": eng.E * world,
                "seq_len": cfg.model.history,
                "parallelism": f"dp{world}",
                "dp_gradient_sync": ("none" if world == 1 else
                                     "all-reduce overlapped with next step (1-step delayed)" if cfg.engine.dp_overlap
                                     else "sync all-reduce every step"),
                "envs_per_gpu": eng.E,
                "hip_graph": use_graph,
                "graph_steps": cfg.engine.graph_steps if use_graph else None,
                "kernel_chunk": eng.chunk,
                "step_kernel": getattr(eng, "step_kernel", None),
                "chunk_schedule": getattr(eng, "chunk_schedule", "static"),
                "learning_knobs": {"target_every": cfg.agent.target_every, "double_dqn": cfg.agent.double_dqn,
                                   "reward_scale": cfg.agent.reward_scale, "ramp_mode": cfg.agent.ramp_mode},
            },
            "graph_prime_steps": prime_steps,
            "world_size": world,
            # one optimizer update per step (sync DP: one global update over every rank's envs)
            "updates_per_s": round(args.steps / el, 1),
            "samples_per_update": eng.E * world,
            "window_return_mean": round(float(ret[0] / ret[1]), 4),
            "window_return_steps": args.steps,
            "mean_reward_per_step": st[0] / max(n_trans, 1),
            "mean_td_loss": st[1] / max(n_trans, 1),
            "vs_reference_floor": round(value / REFERENCE_FLOOR, 1),
        }
        if torch.cuda.is_available():
            free, total = torch.cuda.mem_get_info(eng.device)
            out["hbm_used_gb"] = round((total - free) / 1e9, 1)
            out["hbm_total_gb"] = round(total / 1e9, 1)
            out["alloc_peak_gb_per_rank"] = [round(float(p_[0]), 2) for p_ in peaks]
        if allreduce_ms is not None:
            out["allreduce_ms_per_step"] = allreduce_ms
        if episode_error is not None:
            out["episode_return_error"] = episode_error
        if episodes is not None:
            lr_ = episodes["learned"]
            er = {
                "what": "final portfolio - initial budget, one complete episode per env (untimed, after the "
                        "timed window), mean / population std over all envs of all ranks. greedy: the learned "
                        "parameters frozen, exploit-only; init_greedy: the same at the random init; buy_hold: "
                        "Buy every step (budget into shares, then held); learned: online epsilon-greedy episode "
                        "with learning on; greedy_trained: greedy + frozen with the parameters after that online "
                        "episode; random: uniform actions. median: exact at one rank, the mean of the ranks' "
                        "medians at several",
                "episode_steps": lr_["steps"],
            }
            for k in ("greedy", "init_greedy", "buy_hold", "learned", "greedy_trained", "random"):
                er[f"{k}_mean"] = round(episodes[k]["mean"], 4)
                er[f"{k}_std"] = round(episodes[k]["std"], 4)
                er[f"{k}_median"] = round(episodes[k]["median"], 4)
            er["episodes"] = lr_["n"]
            er["complete_frac"] = round(min(episodes[k]["complete_frac"] for k in episodes), 6)
            if stable is not None:
                if "error" not in stable:
                    stable["greedy_median_minus_random_median"] = round(stable["greedy_median"] -
                                                                        episodes["random"]["median"], 4)
                er["stable_learner"] = stable
            out["episode_return"] = er
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
