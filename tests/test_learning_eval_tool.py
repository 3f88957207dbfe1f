"""tools/learning_eval.py on the CPU (torch backend): one training episode + greedy evaluation + the
init-greedy / buy-and-hold / random baselines on a tiny bank, table written (the tool behind
profiles/r4_learning_*.md)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_learning_eval_runs_on_cpu(tmp_path):
    out = tmp_path / "eval.md"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "learning_eval.py"), "--device", "cpu", "--backend", "torch",
           "--envs", "64", "--length", "260", "--episodes", "1",
           "--run", "t:data.source=trend,agent.target_every=20,agent.double_dqn=true,agent.ramp_mode=global",
           "-o", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    txt = out.read_text()
    assert "## t: data.source=trend" in txt and "buy & hold" in txt and "| 1 |" in txt
