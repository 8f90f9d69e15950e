"""Synthetic workloads shared by the parity tests and bench.py.

Seeded and deterministic: keys id in [0, K), name(id) = b"b" + decimal(id);
Zipf(s) ranks mapped to ids by a fixed multiplicative bijection mod K so hot
keys are scattered; replica states in the clean domain
(taken = f64(U_int[0,1e6)), added = taken + U[0,100), elapsed = U_int[0,2^40)).
"""
from __future__ import annotations

import numpy as np

T0 = 1_700_000_000_000_000_000
SEC = 10**9


def key_names(ids) -> list:
    return [b"b%d" % int(i) for i in ids]


def zipf_ids(rng: np.random.Generator, n: int, K: int, s: float = 1.1) -> np.ndarray:
    """n draws of Zipf(s) over ranks [1, K], scattered over ids by a bijection."""
    ranks = np.arange(1, K + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s)
    cdf /= cdf[-1]
    r = np.searchsorted(cdf, rng.random(n), side="left").astype(np.int64)
    r = np.minimum(r, K - 1)
    mult = 2654435761 % K or 1
    while np.gcd(mult, K) != 1:
        mult += 1
    return (r * mult) % K


def clean_states(rng: np.random.Generator, n: int):
    taken = rng.integers(0, 10**6, n).astype(np.float64)
    added = taken + rng.random(n) * 100.0
    elapsed = rng.integers(0, 1 << 40, n, dtype=np.int64)
    return added.view(np.uint64).copy(), taken.view(np.uint64).copy(), elapsed


SPECIAL_BITS = np.array([0x0, 0x8000000000000000, 0x7FF0000000000000, 0xFFF0000000000000,
                         0x7FF8000000000000, 0xFFF8000000000001, 0x3FF0000000000000,
                         0xBFF0000000000000, 0x0000000000000001, 0x8000000000000001],
                        dtype=np.uint64)


def dirty_states(rng: np.random.Generator, n: int, p_special: float = 0.2):
    """Mostly clean states with -0.0 / NaN / negatives / zeros sprinkled in."""
    a, t, e = clean_states(rng, n)
    for arr in (a, t):
        m = rng.random(n) < p_special
        arr[m] = SPECIAL_BITS[rng.integers(0, len(SPECIAL_BITS), int(m.sum()))]
    z = rng.random(n) < 0.05          # incast requests (IsZero)
    a[z], t[z], e[z] = 0, 0, 0
    neg = rng.random(n) < 0.05
    e[neg] = -e[neg]
    return a, t, e
