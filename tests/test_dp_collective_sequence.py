"""Every rank issues the same collectives in the same order (CPU, gloo, 2 ranks).

A DP run hangs (RCCL) or fails (gloo timeout) the moment one rank issues a collective its peers do not.  This
runs the flow of ``bench.py`` on the torch engine -- parameter broadcast, graph-capture vote, warm-up and timed
steps (one gradient all-reduce each), the evaluation episodes (full episode, random policy, greedy with frozen
weights, buy-and-hold) -- with every ``torch.distributed`` call logged as (op, shape, dtype) between per-step
markers, on two ranks whose price banks differ (no data-dependent collective may appear), and checks the two
logs are identical call for call (``TrainerRouterActor.scala:86-88,137-139``: the broadcast and the gather of
the router, here one collective sequence per step window).
"""
import datetime
import json
import os
import socket
import tempfile

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    log = []

    def wrap(name):
        fn = getattr(dist, name)

        def logged(*a, **k):
            t = a[0] if a else k.get("tensor")
            if isinstance(t, (list, tuple)):
                t = t[0] if t else None
            desc = (name, list(t.shape) if torch.is_tensor(t) else None, str(t.dtype) if torch.is_tensor(t) else None,
                    str(k.get("op", "")))
            log.append(desc)
            return fn(*a, **k)
        setattr(dist, name, logged)

    for name in ("all_reduce", "broadcast", "all_gather", "barrier", "reduce", "all_gather_into_tensor"):
        wrap(name)
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.dtype = "fp32"
    cfg.model.hidden = [16, 16]
    cfg.agent.ramp = 5.0
    E, T = 4, 212
    # rank-dependent banks (and an uneven episode boundary): no collective may depend on the data
    bank = torch.from_numpy(random_walk(T, 50.0 + 10 * rank, 0.02 * (1 + rank), 3 + rank,
                                        n_series=E).astype(np.float32))
    eng = VectorEngine(cfg, prices=bank, device=torch.device("cpu"), rank=rank, world_size=world,
                       group=dist.group.WORLD, envs=E, backend="torch")
    orig_step = eng.step

    def step():
        log.append(("step", eng.step_count))
        orig_step()
    eng.step = step
    eng.sync_params_from(0)
    use_graph, _ = benchkit.prepare_steps(eng, True, rank, world, dist.group.WORLD, eager_prime=2,
                                          log=lambda m: None)
    eng.run(3)      # warm-up
    eng.run(5)      # "timed"
    log.append(("phase", "evaluation"))
    out = {"online": benchkit.full_episode_returns(eng, world, dist.group.WORLD),
           "random": benchkit.full_episode_returns(eng, world, dist.group.WORLD, random_policy=True),
           "greedy": benchkit.greedy_episode_returns(eng, world, dist.group.WORLD),
           "buy_hold": benchkit.buy_and_hold_returns(eng, world, dist.group.WORLD)}
    dist.barrier()
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump({"log": log, "use_graph": use_graph, "out": out}, f, default=str)
    dist.destroy_process_group()


def test_every_rank_issues_the_same_collectives():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d), nprocs=world, join=True, start_method="spawn")
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(world)]
    logs = [r["log"] for r in res]
    n_coll = sum(1 for e in logs[0] if e[0] not in ("step", "phase"))
    assert n_coll > 20, logs[0]                      # the flow really issued collectives
    steps = sum(1 for e in logs[0] if e[0] == "step")
    assert steps > 2 * (212 - 201), steps           # training steps + the evaluation episodes
    for i, (a, b) in enumerate(zip(logs[0], logs[1])):
        assert a == b, (i, a, b)
    assert len(logs[0]) == len(logs[1])
    # every step window holds the same collectives on both ranks, and the reduced results agree
    assert res[0]["use_graph"] == res[1]["use_graph"]
    for k in ("online", "random", "greedy", "buy_hold"):
        assert res[0]["out"][k]["n"] == res[1]["out"][k]["n"], k
        assert abs(res[0]["out"][k]["mean"] - res[1]["out"][k]["mean"]) < 1e-9, k
