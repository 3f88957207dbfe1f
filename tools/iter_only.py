#!/usr/bin/env python3
"""Run only the captured iterations of config 4 (``deep``) or config 5 (``gru``) at their benches' default
shapes, for a kernel timeline of the iteration itself (the benches end with act-alone / update-alone phases,
which is what ``rocprofv3 ... --last N`` would otherwise show).

    rocprofv3 --kernel-trace -d gpurun_out/x -o run -- python3 tools/iter_only.py gru --iters 12
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=("deep", "gru"))
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--k", type=int, default=4, help="iterations per graph")
    a = ap.parse_args()
    import build

    build.build_all()
    from sharetrade.config import preset_config

    dev = torch.device("cuda", 0)
    if a.which == "deep":
        from sharetrade.trainer.deep import DeepDQN

        cfg = preset_config("flagship")
        cfg.model.hidden = [1024] * 4
        cfg.agent.lr = 1e-4
        d = DeepDQN(cfg, dev, envs=16384, batch=4096, replay_capacity=1 << 20, overlap_act=True)
        for _ in range(4):
            d.act_step()
    else:
        from sharetrade.trainer.recurrent import RecurrentDQN

        d = RecurrentDQN(preset_config("recurrent"), dev, envs=65536, seq=16, batch=1024, bars=4096,
                         replay_segments=1 << 17, overlap_act=True)
        for _ in range(4):
            d.act()
    d.capture(iters_per_graph=a.k)
    d.iterations(2 * a.k)
    torch.cuda.synchronize()
    d.iterations(a.iters)
    torch.cuda.synchronize()
    print("ok", a.which, d.updates)


if __name__ == "__main__":
    main()
