"""Command line: ``python -m sharetrade <command>``.

Commands
--------
``train``   run the ShareTradeHelper application (`ShareTradeHelper.scala`):
            price service -> router -> workers -> learner; prints avg/std.
``engine``  run the vectorised engine directly for N steps and print metrics.
``config``  print the resolved configuration (JSON).

Common flags: ``--preset {reference_compat,intended,flagship,test}``,
``--config file.{json,toml}``, ``--set section.key=value`` (repeatable).
"""
from __future__ import annotations

import argparse
import json
import logging
import sys

from .config import Config, preset_config


def _cfg(a) -> Config:
    cfg = Config.load(a.config, a.preset) if a.config else preset_config(a.preset)
    if a.set:
        cfg.override(a.set)
    return cfg


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="sharetrade")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("train", "engine", "config"):
        p = sub.add_parser(name)
        p.add_argument("--preset", default="reference_compat")
        p.add_argument("--config", default=None)
        p.add_argument("--set", action="append", default=[])
        if name == "train":
            p.add_argument("--engine", choices=["actors", "vector"], default="actors")
            p.add_argument("--device", default=None)
            p.add_argument("--max-prices", type=int, default=None, help="truncate the series (smoke runs)")
        if name == "engine":
            p.add_argument("--steps", type=int, default=100)
            p.add_argument("--envs", type=int, default=None)
            p.add_argument("--device", default="auto")
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    logging.basicConfig(level=getattr(logging, cfg.log.loglevel, logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s %(message)s")
    if a.cmd == "config":
        print(cfg.to_json())
        return 0
    if a.cmd == "train":
        from .app import run

        res = run(cfg, engine=a.engine, device=a.device, max_prices=a.max_prices)
        print(json.dumps(res))
        return 0 if res.get("completed") else 1
    if a.cmd == "engine":
        import time

        import torch

        from .trainer.engine import VectorEngine, resolve_device

        dev = resolve_device(a.device)
        eng = VectorEngine(cfg, device=dev, envs=a.envs)
        t0 = time.perf_counter()
        eng.run(a.steps)
        eng.synchronize()
        dt = time.perf_counter() - t0
        out = {"backend": eng.backend, "kernel": getattr(eng, "kernel", None), "envs": eng.E, "steps": a.steps,
               "env_steps_per_s": eng.E * a.steps / dt, **eng.stats_dict(), **eng.portfolio_summary()}
        print(json.dumps(out))
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
