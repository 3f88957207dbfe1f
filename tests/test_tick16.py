"""The 16-bit tick grid of the synthetic price banks (data.prices.tick16_quantize, the host mirror of
csrc/series.hip tick16_kernel): what the flagship kernel's u16 window path relies on."""
import numpy as np

from sharetrade.data.prices import random_walk, tick16_quantize


def _fma32(a, b, c):
    # fma(a, b, c) in fp32: a * b of two floats is exact in float64, + c (= -1 near a * b ~ 1) too: one rounding
    return (a.astype(np.float64) * b.astype(np.float64) + c).astype(np.float32)


def _grid(q):
    m = q.max(axis=1)
    x = np.frexp(m)[1] - 16
    x = np.where(np.ldexp(m, -x) > 65535, x + 1, x)
    return x


def test_quantized_rows_are_ticks_of_one_power_of_two():
    p = random_walk(600, 50.0, 0.03, 5, n_series=64).astype(np.float32)
    p[3] *= 1e-3      # very different scales per row
    p[4] *= 1e4
    q = tick16_quantize(p)
    assert q.dtype == np.float32 and q.shape == p.shape
    for r in range(p.shape[0]):
        m = q[r].max()
        x = np.frexp(m)[1] - 16
        if np.ldexp(m, -x) > 65535:
            x += 1
        t = np.ldexp(q[r], -x)
        assert np.all(t == np.rint(t)) and t.min() >= 1 and t.max() <= 65535
        assert t.max() > 32767          # the smallest exponent that fits: the top tick uses all 16 bits
        # one tick is at most 2^-16 of the row's largest price
        assert np.abs(q[r] - p[r]).max() <= np.ldexp(np.float32(1.0), x - 1) * 1.0000001
    assert np.array_equal(tick16_quantize(q), q)      # already on the grid: unchanged


def test_relative_features_from_ticks_are_bit_identical():
    """w / last - 1 as the kernels compute it (fma(w, rn(1 / last), -1), fp32) is the same number from the ticks
    as from the prices: the power of two cancels exactly."""
    q = tick16_quantize(random_walk(400, 50.0, 0.02, 9, n_series=32).astype(np.float32))
    for r in range(q.shape[0]):
        m = q[r].max()
        x = np.frexp(m)[1] - 16
        if np.ldexp(m, -x) > 65535:
            x += 1
        t = np.ldexp(q[r], -x).astype(np.float32)
        for last in (200, 250, 399):
            fp = _fma32(q[r, : last + 1], np.float32(1.0) / q[r, last], -1.0)
            ft = _fma32(t[: last + 1], np.float32(1.0) / t[last], -1.0)
            assert np.array_equal(fp, ft)


def test_engine_synthetic_bank_is_on_the_grid():
    import torch

    from sharetrade.config import preset_config
    from sharetrade.trainer.engine import VectorEngine

    cfg = preset_config("flagship")
    cfg.engine.dtype = "fp32"
    cfg.data.length = 300
    eng = VectorEngine(cfg, device=torch.device("cpu"), backend="torch", envs=16)
    b = eng.prices.numpy()
    assert np.array_equal(tick16_quantize(b), b)
    cfg.data.tick16 = False
    eng = VectorEngine(cfg, device=torch.device("cpu"), backend="torch", envs=16)
    assert not np.array_equal(tick16_quantize(eng.prices.numpy()), eng.prices.numpy())
