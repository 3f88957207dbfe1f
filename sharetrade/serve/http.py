"""HTTP front end of the policy server (FastAPI): ``python -m sharetrade serve``.

Routes (JSON):

* ``POST /selection_action`` ``{"current_state": [203 floats], "step": s}`` -> ``{"action": "Buy"|"Sell"|"Hold",
  "index": i}`` -- the reference's ``SelectionAction`` message (``QDecisionPolicyActor.scala:32,56-62``),
  one request per call, grouped with concurrent calls by the :class:`DynamicBatcher`;
* ``POST /select`` ``{"states": [[...], ...], "steps": [...] | null, "return_q": bool}`` -> ``{"actions": [...],
  "q": [[...]]}`` -- a whole batch in one launch (``steps`` null = greedy);
* ``POST /select_bin`` -- the binary form for high-rate clients: the body is little-endian float32
  rows of H + 3 values (the H + 2 state values, then the step; step < 0 = greedy), the reply is one
  int8 action per row.  A single-row call goes through the batcher like ``/selection_action``; JSON
  parsing of 203-float lists is what bounds the JSON routes (``profiles/r2_serve_http.md``);
* ``POST /load`` ``{"checkpoint": path}`` -> swaps in the weights of an engine checkpoint; the path is
  resolved under the server's checkpoint root (``ckpt_root``, ``--ckpt-root``) and anything outside it
  is refused (403); without a root the route is disabled;
* ``GET /health`` -> backend, device, served batches / requests;
* ``GET /metrics`` -> Prometheus text format: requests / batches / errors per route, request latency
  histogram, batch-size histogram of the dynamic batcher (one registry per app).
"""
from __future__ import annotations

import asyncio
import os
import time
from typing import List, Optional

import torch
from fastapi import Request
from pydantic import BaseModel

from ..protocol import action_of
from .server import DynamicBatcher, PolicyServer


def load_checkpoint_params(path: str, averaged: bool = True) -> torch.Tensor:
    """Flat fp32 params to serve from an engine checkpoint (``params_ema`` when present and ``averaged``,
    else ``params``):
    a ``.stck`` file, a ``CheckpointManager`` directory (latest file) or a sharded multi-rank directory
    (rank 0 of the newest committed step)."""
    from ..persist.checkpoint import CheckpointManager, load

    if os.path.isdir(path):
        from ..parallel.dp_train import committed_steps

        steps = committed_steps(path)
        if steps:
            path = os.path.join(path, f"step-{steps[-1]:09d}", "rank-0.stck")
        else:
            latest = CheckpointManager(path).latest()
            if latest is None:
                raise FileNotFoundError(f"no checkpoint under {path}")
            path = latest
    state, _ = load(path)
    if "params" not in state:
        raise KeyError(f"{path} holds no 'params' tensor (not an engine checkpoint)")
    # the Polyak-averaged weights when the run kept them (engine.ema_decay > 0) and ``averaged``
    return state["params_ema"] if averaged and "params_ema" in state else state["params"]


class SelectionActionReq(BaseModel):
    current_state: List[float]
    step: float = 0.0


class SelectReq(BaseModel):
    states: List[List[float]]
    steps: Optional[List[float]] = None
    return_q: bool = False


class LoadReq(BaseModel):
    checkpoint: str
    averaged: bool = True   # the Polyak average when the checkpoint holds one


MAX_BIN_ROWS = 1 << 20   # /select_bin rows per call (HTTP 413 above): bounds one call's device work


def resolve_under(root: str, path: str) -> str:
    """``path`` (absolute, or relative to ``root``) resolved with symlinks; PermissionError unless it
    lies inside ``root`` -- a client may only name checkpoints the operator put under the root."""
    base = os.path.realpath(root)
    cand = os.path.realpath(path if os.path.isabs(path) else os.path.join(base, path))
    if cand != base and not cand.startswith(base + os.sep):
        raise PermissionError(f"{path!r} is outside the checkpoint root")
    return cand


def select_mixed(server: PolicyServer, x, steps):
    """Actions for rows whose step may be negative (= greedy) or not (= epsilon-greedy at that step):
    greedy rows and drawing rows go in separate launches and are scattered back in row order."""
    import numpy as np

    g = steps < 0
    out = np.empty(x.shape[0], dtype=np.int8)
    if g.any():
        out[g] = server.infer(x[g], None).cpu().numpy().astype(np.int8)
    if (~g).any():
        out[~g] = server.infer(x[~g], steps[~g]).cpu().numpy().astype(np.int8)
    return out


def make_app(server: PolicyServer, batcher: Optional[DynamicBatcher] = None, ckpt_root: Optional[str] = None,
             max_bin_rows: int = MAX_BIN_ROWS):
    import numpy as np
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import Response
    from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Histogram, generate_latest

    app = FastAPI(title="sharetrade policy server")
    reg = CollectorRegistry()
    m_req = Counter("sharetrade_serve_requests", "request rows served", ["route"], registry=reg)
    m_err = Counter("sharetrade_serve_errors", "rejected calls", ["route"], registry=reg)
    m_lat = Histogram("sharetrade_serve_latency_seconds", "call latency", ["route"], registry=reg,
                      buckets=(1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 1e-1, 1.0))
    m_bs = Histogram("sharetrade_serve_batch_rows", "rows per kernel launch (batcher)", registry=reg,
                     buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096, 16384))
    seen = {"batches": 0}

    def _batch_sizes() -> None:   # fold the batcher's new batch sizes into the histogram
        if batcher is not None:
            bs = batcher.batch_sizes
            for n in bs[seen["batches"]:len(bs)]:
                m_bs.observe(n)
            seen["batches"] = len(bs)

    @app.post("/selection_action")
    async def selection_action(req: SelectionActionReq):
        t0 = time.perf_counter()
        if len(req.current_state) != server.H + 2:
            m_err.labels("selection_action").inc()
            raise HTTPException(400, f"policy input size({server.H + 2}) and state({len(req.current_state)}) "
                                     f"size do not match")
        if batcher is not None:
            a = await asyncio.wrap_future(batcher.submit(req.current_state, req.step))
        else:
            a = int(server.infer([req.current_state], [req.step]).cpu()[0])
        m_req.labels("selection_action").inc()
        m_lat.labels("selection_action").observe(time.perf_counter() - t0)
        return {"action": repr(action_of(a)), "index": int(a)}

    @app.post("/select")
    def select(req: SelectReq):
        t0 = time.perf_counter()
        try:
            out = server.infer(req.states, req.steps, return_q=req.return_q)
        except ValueError as e:
            m_err.labels("select").inc()
            raise HTTPException(400, str(e))
        m_req.labels("select").inc(len(req.states))
        m_lat.labels("select").observe(time.perf_counter() - t0)
        if req.return_q:
            acts, q = out
            return {"actions": acts.cpu().tolist(), "q": q.cpu().tolist()}
        return {"actions": out.cpu().tolist()}

    @app.post("/select_bin")
    async def select_bin(request: Request):
        t0 = time.perf_counter()
        body = await request.body()
        W = server.H + 3
        if len(body) == 0 or len(body) % (4 * W) != 0:
            m_err.labels("select_bin").inc()
            raise HTTPException(400, f"body must be float32 rows of {W} values (state + step)")
        if len(body) // (4 * W) > max_bin_rows:
            m_err.labels("select_bin").inc()
            raise HTTPException(413, f"at most {max_bin_rows} rows per call")
        x = np.frombuffer(body, dtype="<f4").reshape(-1, W)
        steps = x[:, W - 1]
        if x.shape[0] == 1 and batcher is not None and float(steps[0]) >= 0.0:
            # one epsilon-greedy row: grouped with concurrent calls (the batcher draws with steps; a
            # greedy row, step < 0, is answered directly below)
            a = await asyncio.wrap_future(batcher.submit(x[0, : W - 1], float(steps[0])))
            out = np.asarray([a], dtype=np.int8)
        else:
            # a launch plus a device sync: off the event loop, so the batcher's futures and /metrics keep
            # being served meanwhile; greedy (step < 0) and drawing rows in separate launches
            out = await asyncio.to_thread(select_mixed, server, np.ascontiguousarray(x[:, : W - 1]), steps.copy())
        m_req.labels("select_bin").inc(x.shape[0])
        m_lat.labels("select_bin").observe(time.perf_counter() - t0)
        return Response(out.tobytes(), media_type="application/octet-stream")

    @app.post("/load")
    def load(req: LoadReq):
        if ckpt_root is None:
            raise HTTPException(403, "checkpoint loading is disabled (start the server with a checkpoint root)")
        try:
            path = resolve_under(ckpt_root, req.checkpoint)
        except PermissionError as e:
            m_err.labels("load").inc()
            raise HTTPException(403, str(e))
        try:
            server.load_params(load_checkpoint_params(path, req.averaged))
        except (OSError, KeyError, ValueError) as e:
            raise HTTPException(400, str(e))
        return {"loaded": req.checkpoint}

    @app.get("/health")
    def health():
        return {"backend": server.backend, "device": str(server.device), "batches": server.batches,
                "requests": server.requests, "params": server.layout.numel}

    @app.get("/metrics")
    def metrics():
        _batch_sizes()
        return Response(generate_latest(reg), media_type=CONTENT_TYPE_LATEST)

    return app
