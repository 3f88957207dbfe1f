"""bench.py driver contract on one GPU: one JSON line with the required keys, whole-job value =
envs x steps / elapsed, and the flagship config it claims (BASELINE.json metric)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract(native_built):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--envs", "8192", "--steps", "40",
                          "--warmup", "4"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for k in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 40 and d["warmup"] == 4 and d["dtype"] == "bf16"
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    c = d["config"]
    assert c["global_batch"] == 8192 and c["parallelism"] == "dp1" and c["seq_len"] == 201
    # value is the whole-job rate implied by ms_per_step
    assert abs(d["value"] - 8192 / (d["ms_per_step"] * 1e-3)) < 0.01 * d["value"]
    # the untimed evaluations: the plain learner's episodes and the stabilised learner's greedy episode
    er = d["episode_return"]
    for k in ("greedy_median", "random_median", "buy_hold_median"):
        assert k in er, k
    sl = er["stable_learner"]
    assert "error" not in sl, sl
    # trained for as many steps as the plain learner before its evaluation (graph priming + warm-up + timed)
    assert sl["preset"] == "flagship_stable" and 44 <= sl["train_steps"] <= d["graph_prime_steps"] + 44 + 64
    assert "greedy_median" in sl
