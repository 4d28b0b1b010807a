"""Synthetic rectified stereo pairs.

L is i.i.d. uniform u8 from a seeded generator (seed 0x5EED + pair index);
R(y, x) = L(y, min(x + d*(y, x), W - 1)) with a piecewise-constant disparity
field d* made of vertical slabs whose values lie in [0, D - 1].  Optional +-n
uniform noise on R (throughput runs only: it breaks the exact known answer).
There is no dataset or network in this environment; every bench and test input
is generated here.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x5EED


def slab_field(W: int, H: int, D: int, rng: np.random.Generator, min_w: int = 24,
               max_w: int = 96) -> np.ndarray:
    """(H, W) int32 disparity field: vertical slabs of random width / value."""
    row = np.empty(W, dtype=np.int32)
    x = 0
    while x < W:
        w = int(rng.integers(min_w, max_w + 1))
        row[x:x + w] = int(rng.integers(0, D))
        x += w
    return np.broadcast_to(row, (H, W)).copy()


def synthetic_pair(W: int, H: int, D: int, pair_index: int = 0, noise: int = 0):
    """Returns (L, R, dstar) as C-contiguous arrays (u8, u8, int32)."""
    rng = np.random.Generator(np.random.PCG64(SEED_BASE + pair_index))
    L = rng.integers(0, 256, size=(H, W), dtype=np.uint8)
    dstar = slab_field(W, H, D, rng)
    xs = np.minimum(np.arange(W, dtype=np.int64)[None, :] + dstar, W - 1)
    R = np.take_along_axis(L, xs, axis=1)
    if noise:
        n = rng.integers(-noise, noise + 1, size=(H, W))
        R = np.clip(R.astype(np.int32) + n, 0, 255).astype(np.uint8)
    return np.ascontiguousarray(L), np.ascontiguousarray(R), dstar


def expected_known_answer(dstar: np.ndarray, w: int) -> np.ndarray:
    """Per pixel, the disparity the matcher must return where the answer is known, else -1.

    Interior pixel x has zero cost at d when every R column x + dx - d of its
    window lies in a slab of value d (then R(y, x+dx-d) = L(y, x+dx) exactly,
    rows included since d* is constant along y).  The smallest such d wins.
    """
    H, W = dstar.shape
    r = (w - 1) // 2
    row = dstar[0]
    exp = np.full(W, -1, dtype=np.int32)
    for x in range(r, W - r):
        for d in np.unique(row):
            if x - r - d < 0:
                continue
            if all(row[x + dx - d] == d for dx in range(-r, r + 1)):
                exp[x] = d if exp[x] < 0 else min(exp[x], d)
    return np.broadcast_to(exp, (H, W))
