#!/usr/bin/env python3
"""Does the learned policy beat simple policies?  Greedy evaluation of the flagship online DQN.

For each run (a price bank plus config overrides) the engine trains for ``--episodes`` online episodes
(every env plays its series once per episode, epsilon-greedy with the exploit ramp, one Adam update per
step over all envs -- the bench's training regime).  After each episode the current parameters are
evaluated on a snapshot of the engine (restored afterwards), one complete episode per env:

* ``greedy``      -- the learned parameters frozen, exploit-only (no exploration, no learning);
* ``ema greedy``  -- the same with the Polyak-averaged parameters (``engine.ema_decay`` > 0 only);

and once per run, on the same banks:

* ``init greedy`` -- the random-init parameters, frozen, exploit-only;
* ``buy & hold``  -- Buy at every step (budget into shares at the start, then held);
* ``random``      -- uniform Buy / Sell / Hold.

Reported: mean and median of (final portfolio - initial budget) over envs.  Geometric banks are
skewed (a few envs multiply their budget), so the median is the robust figure.

    python tools/learning_eval.py --envs 65536 --length 1601 --episodes 5 \\
        --run "rw:data.source=random_walk" --run "ar1:data.source=ar1" --run "trend:data.source=trend" \\
        -o gpurun_out/learning_eval.md
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _returns(eng, ep0):
    st = eng.state
    done = st.episodes > ep0
    fin = (st.last_final.double() - float(eng.cfg.env.budget))[done]
    return fin, float(done.double().mean())


def _summ(fin: torch.Tensor):
    if fin.numel() == 0:
        return math.nan, math.nan
    return float(fin.mean()), float(fin.median())


def evaluate(eng, mode: str, params=None):
    """One episode per env on a snapshot: mode greedy (frozen, exploit-only) or random (online, eps 0)."""
    from sharetrade.trainer import benchkit

    steps = int(eng.T - eng.H)
    with benchkit.evaluation_snapshot(eng):
        if params is not None:
            eng.set_params(params)
        ep0 = benchkit.reset_episodes(eng)
        over = dict(epsilon=math.inf, lr=0.0) if mode == "greedy" else dict(epsilon=0.0)
        with eng.policy_overrides(**over):
            eng.run(steps)
        eng.synchronize()
        fin, frac = _returns(eng, ep0)
    return _summ(fin), frac


def buy_hold(eng):
    c = eng.cfg.env
    P = eng.prices
    H, T = int(eng.H), int(eng.T)
    b = torch.full((P.shape[0],), float(c.budget), dtype=torch.float32, device=P.device)
    sh = torch.zeros(P.shape[0], dtype=torch.int32, device=P.device) + int(c.shares)
    for pos in range(T - H):
        v = P[:, pos + H]
        buy = b >= v
        b = torch.where(buy, b - v, b)
        sh = sh + buy.to(torch.int32)
    fin = (b + sh.to(torch.float32) * P[:, T - 1]).double() - float(c.budget)
    return _summ(fin)


def run_one(name: str, sets, a, device):
    from sharetrade.config import preset_config
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.data.length = a.length
    cfg.override(list(sets))
    eng = VectorEngine(cfg, device=device, envs=a.envs, backend=a.backend)
    init = eng.params.detach().clone()
    if eng.backend == "native":
        eng.capture_graph(warmup=0)
    t0 = time.perf_counter()
    base = {"init greedy": evaluate(eng, "greedy", init)[0], "buy & hold": buy_hold(eng),
            "random": evaluate(eng, "random")[0]}
    rows = []
    steps = int(eng.T - eng.H)
    for ep in range(a.episodes):
        ep0 = benchkit.reset_episodes(eng)
        eng.run(steps)
        eng.synchronize()
        on, _ = _returns(eng, ep0)
        g, frac = evaluate(eng, "greedy")
        r = {"episode": ep + 1, "online": _summ(on), "greedy": g, "greedy_frac": frac}
        if eng.params_ema is not None:
            r["ema greedy"] = evaluate(eng, "greedy", eng.params_ema.detach().clone())[0]
        rows.append(r)
        print(name, r, flush=True)
    return {"name": name, "sets": sets, "base": base, "rows": rows, "seconds": time.perf_counter() - t0,
            "ema": eng.params_ema is not None}


def fmt(x):
    return f"{x[0]:.0f} / {x[1]:.0f}"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--length", type=int, default=1601, help="series length (episode = length - 201 steps)")
    ap.add_argument("--episodes", type=int, default=5)
    ap.add_argument("--run", action="append", default=[], help="name:key=val,key=val (config overrides)")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--backend", default=None, help="engine backend: native (default on a GPU) | torch (the "
                    "oracle; needed for agent.target_every / double_dqn / reward_scale / ramp_mode runs)")
    ap.add_argument("-o", "--out", default="")
    a = ap.parse_args()
    if a.device == "cuda":
        import build as _b

        _b.build_all()
    dev = torch.device(a.device)
    runs = a.run or ["ar1:data.source=ar1"]
    res = []
    for spec in runs:
        name, _, rest = spec.partition(":")
        sets = [s for s in rest.split(",") if s]
        res.append(run_one(name, sets, a, dev))
    lines = [f"# Greedy evaluation of the learned policy: {a.envs} envs, series length {a.length} "
             f"({a.length - 201} steps per episode), {a.episodes} online episodes per run"
             + (f", `{a.backend}` backend" if a.backend else ""), "",
             "Each cell: mean / median over envs of (final portfolio - initial budget $2,400) for one complete "
             "episode.  `online` = the training episode itself (epsilon-greedy ramp, learning on); `greedy` = "
             "the parameters after that episode, frozen, exploit-only, replayed from the start of the series "
             "on a snapshot (`tools/learning_eval.py`).", ""]
    for r in res:
        b = r["base"]
        lines += [f"## {r['name']}: {' '.join(r['sets']) or '(flagship preset)'}", "",
                  f"baselines: init greedy {fmt(b['init greedy'])}, buy & hold {fmt(b['buy & hold'])}, "
                  f"random {fmt(b['random'])}  ({r['seconds']:.0f} s)", ""]
        head = ["episode", "online", "greedy"] + (["ema greedy"] if r["ema"] else [])
        lines += ["| " + " | ".join(head) + " |", "|" + "---|" * len(head)]
        for row in r["rows"]:
            cells = [str(row["episode"]), fmt(row["online"]), fmt(row["greedy"])]
            if r["ema"]:
                cells.append(fmt(row["ema greedy"]))
            lines.append("| " + " | ".join(cells) + " |")
        lines.append("")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(txt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
