"""Per-call latency of the batch-1 learner behind QDecisionPolicyActor (reference_compat preset): select
(one SelectionAction: forward + argmax + read-back) and update (one UpdateQ), host wall time per call.

    python tools/learner_latency.py [--n 2000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sharetrade.config import preset_config  # noqa: E402
from sharetrade.policy.learner import QLearner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    lr = QLearner(preset_config("reference_compat"), device=dev)
    rng = np.random.default_rng(0)
    s = torch.from_numpy(rng.random((1, 203), dtype=np.float32))
    ns = torch.from_numpy(rng.random((1, 203), dtype=np.float32))
    for _ in range(50):
        lr.select(s, 5.0)
        lr.update(s, 0.5, ns, None, return_loss=False)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    out = {"device": dev.type, "backend": getattr(lr, "backend", "?")}
    t = time.perf_counter()
    for i in range(a.n):
        lr.select(s, float(i))
    out["select_us"] = round((time.perf_counter() - t) / a.n * 1e6, 1)
    t = time.perf_counter()
    for _ in range(a.n):
        lr.update(s, 0.5, ns, None, return_loss=False)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    out["update_us"] = round((time.perf_counter() - t) / a.n * 1e6, 1)
    t = time.perf_counter()
    for i in range(a.n):
        lr.select(s, float(i))
        lr.update(s, 0.5, ns, None, return_loss=False)
    out["select_plus_update_us"] = round((time.perf_counter() - t) / a.n * 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
