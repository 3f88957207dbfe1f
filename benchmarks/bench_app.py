#!/usr/bin/env python3
"""The reference application end to end (BASELINE.json config 1 shape; `ShareTradeHelper.scala:14-48`).

One run = price service -> router -> 10 backoff-supervised workers -> shared policy actor ->
Completed / GetAvg / GetStd, exactly the reference's flow, timed from ActorSystem start to the
poll that sees ``(Completed, Result, Result)``.  Two back ends behind the same actors/messages:

* ``actors``: every worker runs the reference's per-step SelectionAction / UpdateQ round trips
  against the policy actor (batch-1 semantics; fp32 HIP learner on a GPU);
* ``vector``: the workers are lanes of one VectorEngine (fused HIP step kernel on a GPU).

Prices: the reference's MSFT file when present (``SHARETRADE_MSFT_CSV`` / the reference checkout),
otherwise a synthetic random-walk series of the same length (6,047 rows: 5,846 steps per worker).
BASELINE.md's only throughput figure is the derived floor of >= 58 env-steps/s the reference's
App needs to see completion within its 201 x 5 s poll budget.  Prints one JSON line per engine.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REFERENCE_FLOOR = 58.0   # env-steps/s (derived)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", choices=["actors", "vector", "both"], default="both")
    ap.add_argument("--preset", default="reference_compat")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--max-prices", type=int, default=None, help="truncate the series (smoke runs)")
    ap.add_argument("--poll", type=float, default=0.01, help="App poll interval in s (reference: 5.0)")
    ap.add_argument("--synthetic", action="store_true", help="random-walk series even if the MSFT file exists")
    a = ap.parse_args()
    if a.device != "cpu":
        import build

        build.build_all()
    from sharetrade.app import run
    from sharetrade.config import default_csv_path, preset_config

    cfg = preset_config(a.preset)
    budget_s = cfg.router.poll_rounds * cfg.router.poll_interval_s    # the reference's 201 x 5 s
    cfg.router.poll_interval_s = a.poll
    cfg.router.poll_rounds = int(budget_s / a.poll) + 1
    cfg.env.progress_every = 0
    data = "reference MSFT series (read in place)"
    if a.synthetic or not os.path.exists(default_csv_path()):
        cfg.data.source = "random_walk"
        data = f"synthetic random-walk series, {cfg.data.length} rows (MSFT-file shape)"
    n_rows = a.max_prices or cfg.data.length
    engines = ["actors", "vector"] if a.engine == "both" else [a.engine]
    for eng in engines:
        t0 = time.perf_counter()
        res = run(cfg, engine=eng, device=a.device, max_prices=a.max_prices, quiet=True)
        wall = time.perf_counter() - t0
        steps_per_worker = max(n_rows - cfg.model.history, 0)
        env_steps = steps_per_worker * cfg.router.n_workers
        el = res["elapsed_s"]
        out = {
            "metric": "reference application end to end: env steps/s (10 workers, one shared learner)",
            "engine": eng, "preset": a.preset, "device": a.device, "data": data,
            "completed": bool(res["completed"]), "avg": res.get("avg"), "std": res.get("std"),
            "workers": cfg.router.n_workers, "steps_per_worker": steps_per_worker, "env_steps": env_steps,
            "learner_round_trips": 2 * env_steps if eng == "actors" else None,
            "elapsed_s": round(el, 3), "wall_s_incl_teardown": round(wall, 3),
            "poll_interval_s": a.poll,
            "env_steps_per_s": round(env_steps / el, 1) if el > 0 else None,
            "vs_reference_floor": round(env_steps / el / REFERENCE_FLOOR, 1) if el > 0 else None,
        }
        print(json.dumps(out), flush=True)
        if not res["completed"]:
            sys.exit(1)
        if torch.cuda.is_available():
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
