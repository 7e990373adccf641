"""Seeded synthetic Xe-129 ventilation volumes.

The reference ships no input data, so every benchmark and parity case is built from
this generator.  Layout follows the reference: numpy C-order ``(rows, cols, slices)`` with the
slice axis fastest, exactly as ``Vent_Analysis.openSingleDICOM`` produces it
(``Vent_Analysis.py:179``).

* mask  = union of two ellipsoids (the two lungs)
* image = exp(0.4 (i - R/2) / R) * 200 * mask + Rayleigh(10) noise   (a smooth bias field)
* 6 ventilation defects: spheres (slice axis scaled) inside the mask, intensity x 0.2
* ``vary=True`` (benchmark batches): per-seed lung geometry -- each ellipsoid's semi-axes scaled by
  0.8-1.2 and its centre moved by up to 6 % of the extent (a separate stream, so ``vary=False``
  volumes, which the committed fixtures pin by sha256, are unchanged)
"""
from __future__ import annotations

import hashlib

import numpy as np

__all__ = ["synth_volume", "synth_batch", "volume_digest"]


def synth_volume(R: int, C: int, Z: int, seed: int, vary: bool = False):
    """Return ``(HPvent float32 (R,C,Z), mask float64 0/1 (R,C,Z))`` for one study."""
    R, C, Z, seed = int(R), int(C), int(Z), int(seed)   # python ints: numpy scalars change promotion
    rng = np.random.default_rng(seed)
    i, j, k = np.meshgrid(np.arange(R, dtype=np.float32), np.arange(C, dtype=np.float32),
                          np.arange(Z, dtype=np.float32), indexing="ij")
    m = np.zeros((R, C, Z), bool)
    geo = np.random.default_rng(seed + 1_000_003) if vary else None
    for cc in (0.32, 0.68):
        sa, sc, sz = geo.uniform(0.8, 1.2, 3) if vary else (1.0, 1.0, 1.0)
        da, dc, dz = geo.uniform(-0.06, 0.06, 3) if vary else (0.0, 0.0, 0.0)
        m |= (((i - (0.5 + da) * R) / (0.35 * sa * R)) ** 2 + ((j - (cc + dc) * C) / (0.17 * sc * C)) ** 2
              + ((k - (0.5 + dz) * Z) / (0.42 * sz * Z)) ** 2) <= 1
    X = np.exp(0.4 * (i - R / 2) / R) * 200 * m + rng.rayleigh(10, (R, C, Z))
    for _ in range(6):
        c = [rng.uniform(0.2, 0.8) * s for s in (R, C, Z)]
        r = rng.uniform(0.03, 0.08) * R
        d = ((i - c[0]) ** 2 + (j - c[1]) ** 2 + ((k - c[2]) * (R / Z) * 0.2) ** 2 <= r ** 2) & m
        X[d] *= 0.2
    return X.astype(np.float32), m.astype(np.float64)


def synth_batch(R: int, C: int, Z: int, n: int, base_seed: int = 0, unique: int | None = None,
                vary: bool = False):
    """Batch of ``n`` volumes as contiguous ``float32 [n,R,C,Z]`` and ``uint8 [n,R,C,Z]``.

    Volume b uses seed ``base_seed + (b % unique)``: ``unique`` bounds host generation time for
    large benchmark batches (every volume is still processed independently on the device).
    """
    u = n if unique is None else max(1, min(unique, n))
    hp = np.empty((n, R, C, Z), np.float32)
    mk = np.empty((n, R, C, Z), np.uint8)
    cache = {}
    for b in range(n):
        s = base_seed + (b % u)
        if s not in cache:
            x, m = synth_volume(R, C, Z, s, vary)
            cache[s] = (x, m.astype(np.uint8))
        hp[b], mk[b] = cache[s]
    return hp, mk


def volume_digest(*arrays) -> str:
    """sha256 over the raw bytes of the arrays (fixture drift check)."""
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
