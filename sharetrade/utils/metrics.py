"""Metrics / observability.

The reference's only visibility is log lines (progress every 200 steps,
`TrainerChildActor.scala:105-109`) and the final mean/std.  The engine adds a
JSONL metrics stream — env-steps/s (per GPU and whole job), updates/s, mean
reward, TD loss, exploration rate, completed episodes with final-portfolio
mean/std, and the DP all-reduce share — plus optional Chrome traces
(``torch.profiler``) for host/device spans.
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional


class MetricsLogger:
    def __init__(self, path: Optional[str] = None, stdout_every: int = 0):
        self.path = path
        self.f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
            self.f = open(path, "a", buffering=1)
        self.stdout_every = stdout_every
        self.n = 0

    def log(self, record: Dict[str, Any]) -> None:
        rec = {"ts": round(time.time(), 3), **record}
        line = json.dumps(rec, default=float)
        if self.f:
            self.f.write(line + "\n")
        self.n += 1
        if self.stdout_every and self.n % self.stdout_every == 0:
            print(line, flush=True)

    def close(self) -> None:
        if self.f:
            self.f.close()
            self.f = None


class WindowStats:
    """Differences of the engine's running statistics over a logging window."""

    def __init__(self):
        self.prev: Optional[Dict[str, float]] = None
        self.t_prev = time.perf_counter()
        self.step_prev = 0

    def window(self, stats: Dict[str, float], step: int, envs: int, world: int = 1) -> Dict[str, float]:
        now = time.perf_counter()
        cur = dict(stats)
        prev = self.prev or {k: 0.0 for k in cur}
        d = {k: cur.get(k, 0.0) - prev.get(k, 0.0) for k in cur}
        steps = max(1, step - self.step_prev)
        dt = max(1e-9, now - self.t_prev)
        trans = steps * envs
        done = d.get("episodes_done", 0.0)
        out = {
            "step": step,
            "updates_per_s": steps / dt,
            "env_steps_per_s_gpu": trans / dt,
            "env_steps_per_s_job": trans * world / dt,
            "mean_reward": d.get("reward_sum", 0.0) / trans,
            "mean_td_loss": d.get("loss_sum", 0.0) / trans,
            "explore_rate": d.get("explore", 0.0) / trans,
            "episodes_done": done,
        }
        if done > 0:
            m = d.get("final_sum", 0.0) / done
            out["final_portfolio_mean"] = m
            out["final_portfolio_std"] = max(0.0, d.get("final_sq", 0.0) / done - m * m) ** 0.5
        self.prev, self.t_prev, self.step_prev = cur, now, step
        return out
