"""Command line: ``python -m sharetrade <command>``.

Commands
--------
``train``   run the ShareTradeHelper application (`ShareTradeHelper.scala`):
            price service -> router -> workers -> learner; prints avg/std.
``engine``  run the vectorised engine directly for N steps and print metrics.
``deep``    train the 4x1024-MLP replay DQN (BASELINE config 4) for N iterations.
``recurrent`` train the GRU(256) minute-bar DQN (BASELINE config 5) for N iterations.
``serve``   serve SelectionAction over HTTP from the batched GPU kernel (weights from an
            engine checkpoint or random init).
``config``  print the resolved configuration (JSON).

Common flags: ``--preset {reference_compat,intended,flagship,flagship_stable,test}``,
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
    for name in ("train", "engine", "deep", "recurrent", "serve", "config"):
        p = sub.add_parser(name)
        p.add_argument("--preset", default={"deep": "flagship", "recurrent": "recurrent",
                                            "serve": "flagship"}.get(name, "reference_compat"))
        p.add_argument("--config", default=None)
        p.add_argument("--set", action="append", default=[])
        if name == "train":
            p.add_argument("--engine", choices=["actors", "vector"], default="actors")
            p.add_argument("--device", default=None)
            p.add_argument("--max-prices", type=int, default=None, help="truncate the series (smoke runs)")
            p.add_argument("--gpus", type=int, default=1,
                           help="--engine vector: N > 1 makes the router's N routees the ranks of a data-parallel "
                                "group, one process per GPU (RCCL), with rank death -> replacement -> resume")
            p.add_argument("--envs-per-rank", type=int, default=None, help="envs of each rank (--gpus > 1)")
            p.add_argument("--dist-backend", default=None, help="nccl (= RCCL, GPUs) | gloo")
            p.add_argument("--ckpt-dir", default=None, help="--gpus > 1: sharded checkpoints of the episode")
            p.add_argument("--ckpt-every", type=int, default=0)
            p.add_argument("--same-device", action="store_true", help="--gpus > 1: every rank on cuda:0 (rehearsal)")
        if name == "engine":
            p.add_argument("--steps", type=int, default=100)
            p.add_argument("--envs", type=int, default=None)
            p.add_argument("--device", default="auto")
            p.add_argument("--metrics", default=None, help="JSONL metrics output path")
            p.add_argument("--log-every", type=int, default=100)
            p.add_argument("--ckpt-dir", default=None)
            p.add_argument("--ckpt-every", type=int, default=0)
            p.add_argument("--resume", action="store_true")
            p.add_argument("--trace", default=None, help="Chrome trace output path (torch.profiler)")
            p.add_argument("--no-graph", action="store_true")
        if name in ("engine", "deep", "recurrent"):
            p.add_argument("--elastic", type=int, default=0,
                           help="N > 0: run N rank processes under the elastic launcher (heartbeat + progress "
                                "watchdog, whole-generation respawn, resume from committed checkpoints)")
            p.add_argument("--max-restarts", type=int, default=3)
            p.add_argument("--stall-timeout", type=float, default=120.0, help="--elastic: seconds without progress")
            p.add_argument("--pg-timeout", type=float, default=120.0, help="--elastic: collective timeout (s)")
            p.add_argument("--final-dir", default=None, help="each rank writes its final state here")
            p.add_argument("--same-device", action="store_true", help="--elastic: every rank on cuda:0 (rehearsal)")
            if name == "engine":
                p.add_argument("--dist-backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
        if name in ("deep", "recurrent"):
            p.add_argument("--iterations", type=int, default=200)
            p.add_argument("--envs", type=int, default=None)
            p.add_argument("--batch", type=int, default=None)
            if name == "deep":
                p.add_argument("--hidden", default="1024,1024,1024,1024", help="hidden widths (config 4: 4x1024)")
            p.add_argument("--metrics", default=None, help="JSONL metrics output path")
            p.add_argument("--log-every", type=int, default=50)
            p.add_argument("--ckpt-dir", default=None)
            p.add_argument("--ckpt-every", type=int, default=0)
            p.add_argument("--resume", action="store_true")
            p.add_argument("--no-graph", action="store_true")
            p.add_argument("--dist-backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
            p.add_argument("--trace", default=None, help="Chrome trace output path (torch.profiler)")
        if name == "serve":
            p.add_argument("--ckpt", default=None, help="engine checkpoint file or directory (default: random init)")
            p.add_argument("--ckpt-root", default=None,
                           help="directory POST /load may read checkpoints from (default: the --ckpt directory; "
                                "without either, /load is disabled)")
            p.add_argument("--host", default="127.0.0.1")
            p.add_argument("--port", type=int, default=8000)
            p.add_argument("--device", default="auto")
            p.add_argument("--max-batch", type=int, default=4096)
            p.add_argument("--max-delay-us", type=float, default=200.0)
            p.add_argument("--weights", choices=["average", "live"], default="average",
                           help="with a checkpoint that keeps a Polyak average (engine.ema_decay): serve it or the "
                                "live weights (profiles/r2_serve_eval.md: evaluate both)")
    a = ap.parse_args(argv)
    cfg = _cfg(a)
    logging.basicConfig(level=getattr(logging, cfg.log.loglevel, logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s %(message)s")
    if a.cmd == "config":
        print(cfg.to_json())
        return 0
    if a.cmd == "train":
        from .app import run

        dp = None
        if a.gpus > 1:
            dev = a.device or "cuda"
            dp = dict(device="cpu" if dev.startswith("cpu") else "cuda", backend=a.dist_backend,
                      envs_per_rank=a.envs_per_rank or cfg.engine.envs_per_rank, ckpt_dir=a.ckpt_dir,
                      ckpt_every=a.ckpt_every, same_device=a.same_device)
        res = run(cfg, engine=a.engine, device=a.device, max_prices=a.max_prices, gpus=a.gpus, dp=dp)
        print(json.dumps(res, default=str))
        return 0 if res.get("completed") else 1
    if a.cmd in ("engine", "deep", "recurrent") and a.elastic:
        # the launcher never touches the GPU: one fresh process per rank (parallel/elastic_cli.py)
        from .parallel.elastic_cli import run_elastic

        dev = getattr(a, "device", None) or "cuda"
        dev = "cpu" if dev.startswith("cpu") else "cuda"
        kw = dict(device=dev, backend=a.dist_backend, metrics=a.metrics, log_every=a.log_every, ckpt_dir=a.ckpt_dir,
                  ckpt_every=a.ckpt_every, graph=not a.no_graph, final_dir=a.final_dir, pg_timeout_s=a.pg_timeout,
                  same_device=a.same_device)
        if a.cmd == "engine":
            kw.update(steps=a.steps, envs=a.envs)
        else:
            lk = {}
            if a.cmd == "deep":
                lk["hidden"] = [int(x) for x in a.hidden.split(",")]
            if a.envs:
                lk["envs"] = a.envs
            if a.batch:
                lk["batch"] = a.batch
            kw.update(steps=a.iterations, learner_kw=lk)
        import os
        import tempfile

        fd, kw["result_path"] = tempfile.mkstemp(suffix=".json")
        os.close(fd)
        r = run_elastic(a.cmd, cfg, a.elastic, kw, max_restarts=a.max_restarts, stall_timeout_s=a.stall_timeout)
        out = {"ok": r.ok, "restarts": r.restarts, "flagged": r.flagged,
               "generations": [{"generation": g.generation, "exitcodes": g.exitcodes, "ok": g.ok,
                                "seconds": round(g.seconds, 2)} for g in r.generations]}
        try:
            with open(kw["result_path"]) as f:
                out["result"] = json.loads(f.read() or "null")
        except (OSError, ValueError):
            pass
        os.unlink(kw["result_path"])
        print(json.dumps(out, default=str))
        return 0 if r.ok else 1
    if a.cmd in ("deep", "recurrent"):
        import torch

        from .trainer.runs import run as run_learner

        kw = {}
        if a.cmd == "deep":
            kw["hidden"] = [int(x) for x in a.hidden.split(",")]
        if a.envs:
            kw["envs"] = a.envs
        if a.batch:
            kw["batch"] = a.batch
        from .parallel import dist as D

        # under torch.distributed.run: one rank per GPU, synchronous data parallel over RCCL
        ctx = D.init(backend=a.dist_backend, device="cuda")
        res = run_learner(a.cmd, cfg, a.iterations, device=ctx.device, metrics_path=a.metrics,
                          log_every=a.log_every, ckpt_dir=a.ckpt_dir, ckpt_every=a.ckpt_every, resume=a.resume,
                          graph=not a.no_graph, ctx=ctx, trace_path=a.trace, **kw)
        if ctx.is_main:
            print(json.dumps(res, default=float))
        D.shutdown(ctx)
        return 0
    if a.cmd == "serve":
        import uvicorn

        from .serve import DynamicBatcher, PolicyServer
        from .serve.http import load_checkpoint_params, make_app
        from .trainer.engine import resolve_device

        params = load_checkpoint_params(a.ckpt, averaged=a.weights == "average") if a.ckpt else None
        srv = PolicyServer(cfg, params=params, device=resolve_device(a.device))
        bat = DynamicBatcher(srv, max_batch=a.max_batch, max_delay_us=a.max_delay_us)
        try:
            import os

            root = a.ckpt_root or (None if not a.ckpt else
                                   a.ckpt if os.path.isdir(a.ckpt) else os.path.dirname(os.path.abspath(a.ckpt)))
            uvicorn.run(make_app(srv, bat, ckpt_root=root), host=a.host, port=a.port, log_level="warning")
        finally:
            bat.close()
        return 0
    if a.cmd == "engine":
        from .parallel import dist as D
        from .trainer.engine import resolve_device
        from .trainer.loop import train

        ctx = D.init(backend=a.dist_backend, device=None if a.device == "auto" else a.device)
        dev = ctx.device if ctx.is_distributed or a.device == "auto" else resolve_device(a.device)
        res = train(cfg, a.steps, device=dev, envs=a.envs, metrics_path=a.metrics, log_every=a.log_every,
                    ckpt_dir=a.ckpt_dir, ckpt_every=a.ckpt_every, resume=a.resume, trace_path=a.trace,
                    graph=not a.no_graph, rank=ctx.rank, world_size=ctx.world_size, group=ctx.group)
        if ctx.is_main:
            print(json.dumps(res))
        D.shutdown(ctx)
        return 0
    return 2


if __name__ == "__main__":
    sys.exit(main())
