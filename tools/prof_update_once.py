"""cProfile of the batch-1 learner update's host path (``QLearner.update`` on the GPU, reference_compat
preset): where the ~116 us per UpdateQ went before the thread-per-neuron GEMV (profiles/r3_secondary_benches.md).

    python tools/prof_update_once.py
"""
import cProfile, pstats, sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from sharetrade.config import preset_config
from sharetrade.policy.learner import QLearner
lr = QLearner(preset_config("reference_compat"), device=torch.device("cuda"))
rng = np.random.default_rng(0)
s = torch.from_numpy(rng.random((1, 203), dtype=np.float32)); ns = torch.from_numpy(rng.random((1, 203), dtype=np.float32))
for _ in range(100): lr.update(s, 0.5, ns, None, return_loss=False)
torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable()
for _ in range(2000): lr.update(s, 0.5, ns, None, return_loss=False)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
