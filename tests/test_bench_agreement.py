"""bench.py's multi-rank setup is hang-proof (CPU, gloo, 2 ranks).

Every step of the DP bench holds a gradient all-reduce, so a rank whose HIP-graph capture fails must
not run a different number of steps than its peers (``sharetrade/trainer/benchkit.py``).  A fake
engine counts the all-reduces each rank issues; with a capture failure injected on rank 1
(``SHARETRADE_FAIL_CAPTURE=1``) every rank must fall back to eager steps, issue the same collectives
and finish; without it every rank replays graphs.  The gloo group has a short timeout, so a collective
mismatch fails the test instead of hanging it.  Also: the full-episode return of the torch engine
(one complete episode per env, learned and random policy) on two ranks.
"""
import datetime
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


class _Graph:
    def __init__(self, eng, k):
        self.eng, self.k = eng, k

    def replay(self):
        for _ in range(self.k):
            self.eng._ar()


class _FakeEngine:
    device = torch.device("cpu")
    E = 4

    def __init__(self):
        self.step_count = 0
        self.calls = 0
        self._graph = None
        self._graph_k = None

    def _ar(self):
        import torch.distributed as dist

        t = torch.ones(1)
        dist.all_reduce(t)
        self.calls += 1

    def step(self):
        if self._graph is not None:
            self._graph.replay()
        else:
            self._ar()
        self.step_count += 1

    def run(self, n):
        if self._graph_k is not None:
            g, k = self._graph_k
            for _ in range(n // k):
                g.replay()
                self.step_count += k
            n -= (n // k) * k
        for _ in range(n):
            self.step()

    def capture_graph(self, warmup=0, prime=False):
        for _ in range(warmup):
            self.step()
        self._graph = _Graph(self, 1)
        self._graph_k = (_Graph(self, 16), 16)
        return True

    def prime_graph(self, n):
        for _ in range(n):
            self._graph_k[0].replay()
            self.step_count += 16
        return n


def _worker(rank, world, port, fail, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fail:
        os.environ["SHARETRADE_FAIL_CAPTURE"] = fail
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=20))
    from sharetrade.trainer import benchkit

    eng = _FakeEngine()
    use_graph, prime = benchkit.prepare_steps(eng, True, rank, world, dist.group.WORLD, prime_reps=6,
                                              log=lambda m: None)
    eng.run(5)      # warmup
    eng.run(20)     # "timed"
    dist.barrier()
    counts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(counts, torch.tensor([eng.calls, eng.step_count], dtype=torch.int64))
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{int(use_graph)} {prime} " + " ".join(f"{int(c[0])},{int(c[1])}" for c in counts))
    dist.destroy_process_group()


def _run(fail):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), fail, d), nprocs=world, join=True,
                           start_method="spawn")
        return [open(os.path.join(d, f"r{r}.txt")).read().split() for r in range(world)]


def test_capture_failure_on_one_rank_sends_every_rank_eager():
    res = _run("1")
    for r in res:
        assert r[0] == "0", res                      # nobody replays graphs
        assert len(set(r[2:])) == 1, res            # identical (all-reduce count, step count) on every rank
    assert res[0][1] == res[1][1]                    # same priming on both ranks


def test_no_failure_every_rank_replays_graphs():
    res = _run("")
    for r in res:
        assert r[0] == "1", res
        assert len(set(r[2:])) == 1, res


def _episode_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from sharetrade.config import preset_config
    from sharetrade.data.prices import random_walk
    from sharetrade.trainer import benchkit
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.dtype = "fp32"
    cfg.model.hidden = [16, 16]
    E, T = 6, 215
    bank = torch.from_numpy(random_walk(T, 50.0, 0.02, 5, n_series=E * world).astype(np.float32))
    eng = VectorEngine(cfg, prices=bank[rank * E:(rank + 1) * E], device=torch.device("cpu"), rank=rank,
                       world_size=world, group=dist.group.WORLD, envs=E, backend="torch")
    eng.sync_params_from(0)
    eng.run(3)
    p_before, pos_before = eng.params.clone(), eng.state.pos.clone()
    greedy = benchkit.greedy_episode_returns(eng, world, dist.group.WORLD)
    bh = benchkit.buy_and_hold_returns(eng, world, dist.group.WORLD)
    restored = bool(torch.equal(p_before, eng.params) and torch.equal(pos_before, eng.state.pos))
    learned = benchkit.full_episode_returns(eng, world, dist.group.WORLD)
    rnd = benchkit.full_episode_returns(eng, world, dist.group.WORLD, random_policy=True)
    # the random-policy episode: every action is the uniform draw (exploit prob forced to 0)
    with open(os.path.join(out_dir, f"e{rank}.txt"), "w") as f:
        f.write(f"{learned['n']} {learned['steps']} {learned['mean']!r} {learned['std']!r} "
                f"{rnd['n']} {rnd['mean']!r} {rnd['std']!r} {cfg.agent.epsilon!r} "
                f"{greedy['n']} {greedy['mean']!r} {bh['n']} {bh['mean']!r} {int(restored)} {cfg.agent.lr!r}")
    dist.destroy_process_group()


def test_full_episode_returns_two_ranks():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_episode_worker, args=(world, _free_port(), d), nprocs=world, join=True,
                           start_method="spawn")
        res = [open(os.path.join(d, f"e{r}.txt")).read().split() for r in range(world)]
    assert res[0] == res[1]                          # the reduced statistics agree on every rank
    n, steps, m, s, n_r, m_r, s_r, eps, n_g, m_g, n_bh, m_bh, restored, lr = res[0]
    assert int(n) == 12 and int(steps) == 215 - 201  # every env of both ranks completed one episode
    assert int(n_r) == 12 and int(n_g) == 12 and int(n_bh) == 12
    for v in (m, s, m_r, s_r, m_g, m_bh):
        assert np.isfinite(float(v))
    assert float(eps) == 0.9                         # the epsilon override was restored
    assert restored == "1" and float(lr) == 1e-3     # the greedy evaluation ran on a snapshot


def _vote_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SHARETRADE_FAIL_CAPTURE="1")
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=20))
    from sharetrade.trainer import benchkit

    eng = _FakeEngine()
    use = benchkit.capture_with_vote(eng, rank, world, dist.group.WORLD, warmup=0, log=lambda m: None)
    eng.run(10)
    with open(os.path.join(out_dir, f"v{rank}.txt"), "w") as f:
        f.write(f"{int(use)} {int(eng._graph is None and eng._graph_k is None)} {eng.calls}")
    dist.destroy_process_group()


def test_capture_with_vote_drops_graphs_on_every_rank():
    """The train() / rank-group capture path: rank 1's capture fails, so both ranks drop
    their graphs and step eagerly with the same collectives."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_vote_worker, args=(world, _free_port(), d), nprocs=world, join=True,
                           start_method="spawn")
        res = [open(os.path.join(d, f"v{r}.txt")).read().split() for r in range(world)]
    assert res[0] == res[1] == ["0", "1", "10"], res
