#!/usr/bin/env python3
"""HTTP serving benchmark: ``python -m sharetrade serve`` under concurrent ``SelectionAction`` clients.

Starts the server as a child process (FastAPI + uvicorn, ``DynamicBatcher`` -> ``csrc/qserve.hip``),
waits for ``/health``, then runs ``--clients`` asyncio clients (httpx), each posting ``--requests``
blocking single-row calls in sequence (JSON ``/selection_action`` and binary ``/select_bin``), plus
whole-batch calls (JSON ``/select`` and binary ``/select_bin``) per batch size.
Prints one JSON line per measurement and stops the server (its own PID only).

Synthetic request rows (geometric random-walk prices, random budget / shares); random-init weights.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(B, H=201, seed=0):
    g = np.random.default_rng(seed)
    p = 50.0 * np.exp(np.cumsum(g.normal(0, 0.02, size=(B, H)), axis=1))
    return np.concatenate([p, g.uniform(0, 5000, (B, 1)), g.integers(0, 40, (B, 1))], 1).astype(np.float32)


async def clients(url: str, n: int, per: int, X: np.ndarray, binary: bool):
    import httpx

    lat = []

    async def one(c: int, cl):
        for i in range(per):
            row = X[(c * per + i) % len(X)]
            t = time.perf_counter()
            if binary:
                r = await cl.post(url + "/select_bin", content=np.append(row, np.float32(i)).astype("<f4").tobytes())
            else:
                r = await cl.post(url + "/selection_action", json={"current_state": row.tolist(), "step": float(i)})
            r.raise_for_status()
            lat.append(time.perf_counter() - t)

    limits = httpx.Limits(max_connections=n, max_keepalive_connections=n)
    async with httpx.AsyncClient(timeout=60.0, limits=limits) as cl:
        await one(0, cl)   # warm-up
        lat.clear()
        t0 = time.perf_counter()
        await asyncio.gather(*(one(c, cl) for c in range(n)))
        el = time.perf_counter() - t0
    return lat, el


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", default="1,16,64")
    ap.add_argument("--requests", type=int, default=100, help="per client")
    ap.add_argument("--batches", default="1024,16384")
    args = ap.parse_args()

    import httpx

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    url = f"http://127.0.0.1:{port}"
    srv = subprocess.Popen([sys.executable, "-m", "sharetrade", "serve", "--port", str(port), "--max-delay-us", "200"],
                           cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        for _ in range(600):
            try:
                if httpx.get(url + "/health", timeout=1.0).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.2)
        else:
            raise RuntimeError("server did not come up")
        backend = httpx.get(url + "/health").json()["backend"]
        X = rows(4096)
        for n, binary in [(int(c), b) for c in args.clients.split(",") for b in (False, True)]:
            lat, el = asyncio.run(clients(url, n, args.requests, X, binary))
            us = np.asarray(lat) * 1e6
            print(json.dumps({"bench": "http_select_bin" if binary else "http_selection_action", "backend": backend,
                              "clients": n,
                              "requests": len(lat), "requests_per_s": round(len(lat) / el, 1),
                              "latency_us_p50": round(float(np.percentile(us, 50)), 1),
                              "latency_us_p99": round(float(np.percentile(us, 99)), 1)}), flush=True)
        for B in [int(b) for b in args.batches.split(",")]:
            R = rows(B, seed=B)
            for binary in (False, True):
                if binary:
                    kw = {"content": np.concatenate([R, np.full((B, 1), 500.0, np.float32)], 1).astype("<f4").tobytes()}
                    route = "/select_bin"
                else:
                    kw = {"json": {"states": R.tolist(), "steps": [500.0] * B}}
                    route = "/select"
                httpx.post(url + route, timeout=120.0, **kw).raise_for_status()   # warm-up
                reps = 5
                t = time.perf_counter()
                for _ in range(reps):
                    httpx.post(url + route, timeout=120.0, **kw).raise_for_status()
                el = (time.perf_counter() - t) / reps
                print(json.dumps({"bench": "http_batch" + ("_bin" if binary else "_json"), "backend": backend,
                                  "batch": B, "ms_per_call": round(el * 1e3, 2), "rows_per_s": round(B / el, 1)}),
                      flush=True)
    finally:
        srv.terminate()
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()
            srv.wait(timeout=30)
    return 0


if __name__ == "__main__":
    sys.exit(main())
