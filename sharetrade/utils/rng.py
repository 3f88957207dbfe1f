"""Counter-based Philox4x32-10 RNG — bit-identical host mirror of the device RNG.

The reference draws exploration decisions from the unseeded, stateful
``scala.util.Random`` (`QDecisionPolicyActor.scala:58,62`, quirk Q8).  The
engine instead uses a seeded counter-based generator so that every
(env, step) draw is reproducible, independent of launch geometry, and
identical between this NumPy mirror and `csrc/philox.h`.

Counter layout used by the engine: ``(c0, c1, c2, c3) = (env, step_lo, step_hi, stream)``,
key = ``(seed_lo, seed_hi ^ rank * 0x9E3779B9)``.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32(c0, c1, c2, c3, k0, k1, rounds: int = 10):
    """Vectorised Philox4x32 over uint32 arrays; returns four uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32).copy()
    c1 = np.asarray(c1, dtype=np.uint32).copy()
    c2 = np.asarray(c2, dtype=np.uint32).copy()
    c3 = np.asarray(c3, dtype=np.uint32).copy()
    k0 = np.asarray(k0, dtype=np.uint32).copy()
    k1 = np.asarray(k1, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        for _ in range(rounds):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + W0).astype(np.uint32)
            k1 = (k1 + W1).astype(np.uint32)
    return c0, c1, c2, c3


_SCALAR_MAX = 8
_INV24 = 1.0 / 16777216.0   # (v >> 8) * 2^-24 is exact in fp32 and fp64 alike


def _philox_scalar(c0: int, c1: int, c2: int, c3: int, k0: int, k1: int, rounds: int = 10):
    """Philox4x32 on Python ints (one counter); same bits as :func:`philox4x32`."""
    for _ in range(rounds):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c3 ^ k1) & 0xFFFFFFFF, \
            p0 & 0xFFFFFFFF
        k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
        k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
    return c0, c1, c2, c3


def key_for(seed: int, rank: int = 0):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32(((seed >> 32) ^ (int(rank) * 0x9E3779B9)) & 0xFFFFFFFF)
    return k0, k1


def u24(x) -> np.ndarray:
    """uint32 -> float32 uniform in [0,1) with 24 bits (exact in fp32)."""
    return (np.asarray(x, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def uniforms(seed: int, rank: int, env_ids, step: int, stream: int = 0):
    """Two uniforms per env for the engine's epsilon-greedy draw."""
    k0, k1 = key_for(seed, rank)
    env_ids = np.asarray(env_ids, dtype=np.uint32)
    n = env_ids.shape[0]
    step = int(step)
    c1 = np.full(n, step & 0xFFFFFFFF, dtype=np.uint32)
    c2 = np.full(n, (step >> 32) & 0xFFFFFFFF, dtype=np.uint32)
    c3 = np.full(n, stream, dtype=np.uint32)
    r0, r1, _, _ = philox4x32(env_ids, c1, c2, c3, np.full(n, k0), np.full(n, k1))
    return u24(r0), u24(r1)


class PhiloxStream:
    """Small stateful wrapper (host-side random draws for the actor API path)."""

    def __init__(self, seed: int, rank: int = 0, stream: int = 1):
        self.seed, self.rank, self.stream = seed, rank, stream
        self.counter = 0

    def next_blocks(self, n: int) -> np.ndarray:
        """``n`` independent draws of 4 uniforms (one Philox counter each) -> [n, 4];
        a batch of ``n`` consumes exactly the counters ``n`` single draws would."""
        k0, k1 = key_for(self.seed, self.rank)
        if n <= _SCALAR_MAX:
            # few rows (the actor path's batch-1 SelectionAction): Python-int Philox, bit-identical to the
            # vectorised form -- ~60 numpy calls on 1-element arrays cost 100-250 us per draw, this ~15 us
            out = np.empty((n, 4), dtype=np.float32)
            for j in range(n):
                c = self.counter + j
                r = _philox_scalar(c & 0xFFFFFFFF, (c >> 32) & 0xFFFFFFFF, 0, int(self.stream) & 0xFFFFFFFF,
                                   int(k0), int(k1))
                out[j] = [(v >> 8) * _INV24 for v in r]
            self.counter += n
            return out
        c = np.arange(self.counter, self.counter + n, dtype=np.uint64)
        r = philox4x32((c & np.uint64(0xFFFFFFFF)).astype(np.uint32), (c >> np.uint64(32)).astype(np.uint32),
                       np.zeros(n, np.uint32), np.full(n, self.stream, np.uint32),
                       np.full(n, k0, np.uint32), np.full(n, k1, np.uint32))
        self.counter += n
        return np.stack([u24(v) for v in r], axis=1)

    def next_uniforms(self, n: int = 2) -> np.ndarray:
        out = []
        while len(out) < n:
            k0, k1 = key_for(self.seed, self.rank)
            c = self.counter
            r = philox4x32(np.uint32(c & 0xFFFFFFFF), np.uint32((c >> 32) & 0xFFFFFFFF),
                           np.uint32(0), np.uint32(self.stream), k0, k1)
            self.counter += 1
            out.extend(float(u24(v)) for v in r)
        return np.asarray(out[:n], dtype=np.float32)
