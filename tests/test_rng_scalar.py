"""The host Philox stream's scalar fast path (few rows: the actor path's batch-1 SelectionAction) draws
exactly the bits of the vectorised form -- the oracle tests depend on these draws matching the kernels'."""
import numpy as np

from sharetrade.utils import rng


def _draws(seed, stream, start, sizes, scalar_max):
    old = rng._SCALAR_MAX
    rng._SCALAR_MAX = scalar_max
    try:
        s = rng.PhiloxStream(seed, stream=stream)
        s.counter = start
        return np.concatenate([s.next_blocks(n) for n in sizes]), s.counter
    finally:
        rng._SCALAR_MAX = old


def test_scalar_path_bit_identical():
    for seed, stream, start in ((7, 3, 0), (2 ** 40 + 5, 1, 2 ** 32 - 3), (0, 0, 123456789), (2 ** 63 + 11, 2, 5)):
        sizes = [1] * 9 + [3, 8, 1, 20]
        a, ca = _draws(seed, stream, start, sizes, 8)
        b, cb = _draws(seed, stream, start, sizes, 0)
        assert a.dtype == b.dtype == np.float32
        assert np.array_equal(a, b)
        assert ca == cb == start + sum(sizes)
