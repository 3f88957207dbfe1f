"""Pieces of the flagship benchmark (``bench.py``) that must behave identically on every rank.

A multi-GPU run is one process per GPU over RCCL; every captured or eager step holds a gradient
all-reduce, so every rank must issue the SAME sequence of collectives or the job hangs (the
reference's equivalent invariant: ``router.route(Train(d))`` reaches every routee,
`TrainerRouterActor.scala:86-88`).  Hence:

* :func:`agree` -- a boolean decided by every rank (MIN all-reduce): one rank's failed HIP-graph
  capture sends every rank down the eager path with the same step counts;
* :func:`prepare_steps` -- capture, agree, then prime (graph replays or eager steps: fixed counts on
  every rank);
* :func:`full_episode_returns` -- the headline's "episode return" half: every env plays one complete
  episode over its series (the reference's episode, `TrainerChildActor.scala:64-71`: 6,047 prices ->
  5,846 online-learning steps), final portfolio minus the initial budget, reduced over all ranks
  like the router's ``GetAvg`` / ``GetStd`` (`TrainerRouterActor.scala:89-94,148-151`).
"""
from __future__ import annotations

import contextlib
import math
import os
import sys
from typing import Dict, Optional, Tuple

import torch


def _dist():
    import torch.distributed as dist

    return dist


def agree(ok: bool, world: int, group=None, device: Optional[torch.device] = None) -> bool:
    """True only if ``ok`` on every rank (all-reduce MIN; one collective on every rank)."""
    if world <= 1:
        return bool(ok)
    dist = _dist()
    dev = device if device is not None else torch.device("cpu")
    if dist.get_backend(group) == "gloo":
        dev = torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _fail_capture_here(rank: int) -> bool:
    """Fault injection: ``SHARETRADE_FAIL_CAPTURE=<rank>[,<rank>...]`` makes those ranks' graph
    capture raise (tests of the rank-agreement path)."""
    spec = os.environ.get("SHARETRADE_FAIL_CAPTURE", "")
    return bool(spec) and str(rank) in [s.strip() for s in spec.split(",")]


def prepare_steps(eng, want_graph: bool, rank: int, world: int, group=None, prime_reps: int = 4,
                  eager_prime: int = 64, log=None, fixed_prime: bool = False) -> Tuple[bool, int]:
    """Capture the step graphs (``want_graph``), agree across ranks, then prime.

    Returns ``(use_graph, prime_steps)``.  The 2 eager warm-up steps (each holds an all-reduce) run
    on every rank BEFORE the capture; the capture itself issues no collective (a captured RCCL call
    runs at replay), so a rank whose capture fails has issued exactly the collectives its peers
    have.  The vote follows, then every rank either replays the graphs a fixed number of times or
    runs ``eager_prime`` eager steps: identical collective counts everywhere.  ``fixed_prime``: exactly
    ``prime_reps`` multi-step replays on one rank too (instead of replaying until the clock settles), so
    the number of training steps before the timed window -- and the learned policy the bench evaluates --
    is the same on every run."""
    log = log or (lambda m: print(m, file=sys.stderr))
    start = eng.step_count
    ok = False
    if want_graph:
        eng.run(2)   # eager (no graph captured yet): lazy init of the kernels and the communicator
        try:
            if _fail_capture_here(rank):
                raise RuntimeError("injected capture failure (SHARETRADE_FAIL_CAPTURE)")
            ok = bool(eng.capture_graph(warmup=0, prime=False))
        except Exception as e:  # noqa: BLE001 -- fall back to eager launches, same math
            log(f"rank {rank}: HIP graph capture failed ({str(e).splitlines()[0]})")
            ok = False
        if not ok:
            _drop_graphs(eng)
    use_graph = agree(ok, world, group, getattr(eng, "device", None))
    if not use_graph:
        _drop_graphs(eng)
    if use_graph:
        eng._graph.replay()
        eng.step_count += 1
        if world > 1:
            # a fixed number of multi-step replays on every rank (each replay holds all-reduces)
            gk = getattr(eng, "_graph_k", None)
            if gk is not None:
                for _ in range(max(1, prime_reps)):
                    gk[0].replay()
                    eng.step_count += gk[1]
        else:
            eng.prime_graph(prime_reps, max_reps=prime_reps if fixed_prime else 40)
    else:
        eng.run(eager_prime)
    return use_graph, eng.step_count - start


def capture_with_vote(eng, rank: int, world: int, group=None, warmup: int = 0, log=None) -> bool:
    """Capture ``eng``'s step graphs and agree across ranks (all-reduce MIN) whether to replay them.

    A rank whose capture raises or returns False drops its graphs with ``_drop_graphs`` (the HIP
    runtime's sticky capture error cleared and the device synchronised, so its first eager launch does
    not report the failed capture); if any rank failed, every rank drops its graphs and runs eager
    steps -- the same collectives everywhere.  ``SHARETRADE_FAIL_CAPTURE`` injects the failure."""
    log = log or (lambda m: print(m, file=sys.stderr))
    ok = False
    try:
        if _fail_capture_here(rank):
            raise RuntimeError("injected capture failure (SHARETRADE_FAIL_CAPTURE)")
        ok = bool(eng.capture_graph(warmup=warmup))
    except Exception as e:  # noqa: BLE001 -- eager launches, same math
        log(f"rank {rank}: HIP graph capture failed ({str(e).splitlines()[0] if str(e) else type(e).__name__})")
        ok = False
    if not ok:
        _drop_graphs(eng)
    use = agree(ok, world, group, getattr(eng, "device", None))
    if not use:
        _drop_graphs(eng)
    return use


def _drop_graphs(eng) -> None:
    eng._graph, eng._graph_k = None, None
    if getattr(eng, "device", torch.device("cpu")).type == "cuda":
        try:
            from ..ops import native as _native

            _native.clear_last_error()
        except Exception:  # noqa: BLE001
            pass
        torch.cuda.synchronize()


def reset_episodes(eng) -> torch.Tensor:
    """Every env back to the start of its series with the initial budget / shares; returns the
    per-env completed-episode counters before the reset (to detect completions)."""
    c = eng.cfg.env
    st = eng.state
    st.pos.zero_()
    st.budget.fill_(float(c.budget))
    st.shares.fill_(int(c.shares))
    st.value.zero_()
    st.ret_sum.zero_()
    st.last_final.fill_(float("nan"))
    return st.episodes.clone()


@contextlib.contextmanager
def evaluation_snapshot(eng):
    """Run an evaluation on the engine and put everything back afterwards: parameters, optimizer state,
    step counters, env state and the step-statistics accumulators (an evaluation episode moves the env
    positions, the optimizer moments -- even at lr 0 -- and the statistics)."""
    eng.synchronize()
    snap = eng.state_dict()
    acc = [t.clone() for t in (getattr(eng, "stat_acc", None), getattr(eng, "stats", None)) if torch.is_tensor(t)]
    try:
        yield eng
    finally:
        # no error-word check in here: it would replace an exception raised by the body
        eng.synchronize(check=False)
        eng.load_state_dict(snap)
        for t, c in zip([t for t in (getattr(eng, "stat_acc", None), getattr(eng, "stats", None))
                         if torch.is_tensor(t)], acc):
            t.copy_(c)
        eng.synchronize(check=False)
    eng.check_kernel_err()   # reached only when the body succeeded


def _episode_summary(eng, ep0: torch.Tensor, world: int, group, steps: int) -> Dict[str, float]:
    st = eng.state
    done = st.episodes > ep0
    fin = st.last_final.double() - float(eng.cfg.env.budget)
    fin = torch.where(done, fin, torch.zeros_like(fin))
    return _reduce_returns(done, fin, eng.E, world, group, steps)


def _reduce_returns(done: torch.Tensor, fin: torch.Tensor, E: int, world: int, group, steps: int) -> Dict[str, float]:
    """Mean / population std over every completed env of every rank, and the median: exact with one rank,
    the mean of the ranks' medians with several (a geometric bank's mean is carried by the few series
    that compound; the median is the typical env)."""
    sel = fin[done]
    med = sel.median().double() if sel.numel() else torch.tensor(0.0, dtype=torch.float64, device=fin.device)
    s = torch.stack([done.double().sum(), fin.sum(), (fin * fin).sum(), med.to(fin.device)])
    if world > 1:
        dist = _dist()
        if dist.get_backend(group) == "gloo":
            s = s.cpu()
        dist.all_reduce(s, group=group)
    n, sx, sxx, smed = (float(v) for v in s.cpu())
    n_total = float(E * world)
    if n == 0:
        return {"n": 0, "mean": math.nan, "std": math.nan, "median": math.nan, "steps": steps, "complete_frac": 0.0}
    m = sx / n
    return {"n": int(n), "mean": m, "std": math.sqrt(max(0.0, sxx / n - m * m)), "median": smed / max(1, world),
            "steps": steps, "complete_frac": n / n_total}


def greedy_episode_returns(eng, world: int = 1, group=None, params: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """One complete episode per env with the CURRENT parameters (or ``params``, e.g. the random init)
    frozen and the greedy policy (exploit at every step, no exploration, no learning: the optimizer runs
    at lr 0), on a snapshot of the engine that is restored afterwards.  This measures the learned policy
    itself, without the epsilon-greedy schedule of the online episodes (whose first ~1,000 steps are
    mostly random)."""
    steps = int(eng.T - eng.H)
    with evaluation_snapshot(eng):
        if params is not None:
            eng.set_params(params)
        ep0 = reset_episodes(eng)
        with eng.policy_overrides(epsilon=math.inf, lr=0.0):
            p0 = eng.params.detach().clone()
            eng.run(steps)
            eng.synchronize()
            if not torch.equal(p0, eng.params):
                raise RuntimeError("greedy evaluation changed the parameters (lr 0 expected to freeze them)")
        out = _episode_summary(eng, ep0, world, group, steps)
    return out


def buy_and_hold_returns(eng, world: int = 1, group=None) -> Dict[str, float]:
    """The buy-and-hold baseline on the engine's own price banks, within its action space: Buy at every
    step (one share whenever the budget covers the price, as the env's Buy does), so the budget goes
    into shares at the start of the episode and the position is then held to the end.  Same arithmetic
    as the env step (fp32, one rounding per operation); returns final portfolio - initial budget."""
    c = eng.cfg.env
    P = eng.prices
    H, T = int(eng.H), int(eng.T)
    steps = T - H
    b = torch.full((P.shape[0],), float(c.budget), dtype=torch.float32, device=P.device)
    sh = torch.full((P.shape[0],), int(c.shares), dtype=torch.int32, device=P.device)
    b0 = b.clone()
    s0 = sh.clone()
    for pos in range(steps):
        v = P[:, pos + H]
        # the env's own Buy transition: with env.compat_decisions (TrainerChildActor.scala:120-122) the
        # decision and its update start from the constructor budget / shares at every step, so Buy never
        # accumulates -- the baseline is still "Buy at every step" of THAT env
        bd, sd = (b0, s0) if c.compat_decisions else (b, sh)
        buy = bd >= v
        b = torch.where(buy, bd - v, bd)
        sh = sd + buy.to(torch.int32)
    fin = (b + sh.to(torch.float32) * P[:, T - 1]).double() - float(c.budget)
    done = torch.ones_like(fin, dtype=torch.bool)
    return _reduce_returns(done, fin, P.shape[0], world, group, steps)


def full_episode_returns(eng, world: int = 1, group=None, random_policy: bool = False) -> Dict[str, float]:
    """One complete episode per env (``T - H`` steps, online learning on), then mean / population
    std of (final portfolio - initial budget) over every env of every rank.

    ``random_policy``: the epsilon-greedy exploit probability is forced to 0 for this episode (every
    action uniform over Buy / Sell / Hold, same draws, same banks): the baseline a learned policy has
    to beat.  It runs with eager launches (``policy_overrides``); the learner still updates, which does
    not change a random policy's actions."""
    steps = int(eng.T - eng.H)
    ep0 = reset_episodes(eng)
    if random_policy:
        with eng.policy_overrides(epsilon=0.0):
            eng.run(steps)
    else:
        eng.run(steps)
    eng.synchronize()
    return _episode_summary(eng, ep0, world, group, steps)
