"""Sphere-growing pixel tables for the cluster index (CI.py:33-63, getSpherePix).

The reference builds the table with a 5000-step Python loop over radii (~60 s) and caches it as
``'{v0}x{v1}x{v2}_{R}.npy'`` in the current directory (CI.py:43-61).  This module produces the
*identical* float64 (rows, 4) table [r, dx, dy, dz] in about a second with the same float64
expressions, vectorised:

* ``vox = vox / min(vox)``; ``X, Z, Y = meshgrid(range(-R, R+1))`` (default 'xy' indexing, so the
  row order inside a shell is C-order over that meshgrid: Z, then X, then Y)       CI.py:51-52
* shell ``i`` (r_i = arange(0, R, 0.01)[i]) holds the points with
  ``(r_i - 0.01)^2 < (X v0)^2 + (Y v1)^2 + (Z v2)^2 <= r_i^2``                     CI.py:55-56
  evaluated exactly as the reference does, so a point that rounding puts in two shells (or none)
  appears twice (or not at all), as in the reference table;
* a leading ``[0, 0, 0, 0]`` row                                                      CI.py:53

Parity with the two reference tables is checked bit-for-bit in tests/test_sphere_table.py (sha256
pinned in tests/golden/sphere_tables.json).

``compact_table`` derives what the GPU kernel consumes: int16 offsets, the shell-boundary prefix
lengths of CI.py:79-85 (getRadiiIndices), and a per-row "duplicate linear offset" flag for arrays
so small that two offsets alias to one linear index (CI.py:65-68 px2vec + np.intersect1d's
uniquing, CI.py:96).
"""
from __future__ import annotations

import functools

import numpy as np

__all__ = ["sphere_pix", "radii_indices", "compact_table", "SphereTable"]


@functools.lru_cache(maxsize=8)
def _sphere_pix_cached(vox_key: tuple, radius: int) -> np.ndarray:
    vox = np.divide(np.asarray(vox_key, dtype=np.float64), np.min(vox_key))
    rng = range(-radius, radius + 1, 1)
    X, Z, Y = np.meshgrid(rng, rng, rng)
    d2 = ((X * vox[0]) ** 2 + (Y * vox[1]) ** 2 + (Z * vox[2]) ** 2).ravel()
    rs = np.arange(0, radius, 0.01)
    hi2 = rs ** 2
    lo2 = (rs - 0.01) ** 2
    # candidate first shell: smallest i with r_i^2 >= d2; rounding may also admit i-1 .. i+2
    base = np.searchsorted(hi2, d2, side="left")
    mem_i, mem_p = [], []
    pts = np.arange(d2.size)
    for off in (-1, 0, 1, 2):
        i = base + off
        ok = (i >= 0) & (i < rs.size)
        ii = np.where(ok, i, 0)
        hit = ok & (d2 <= hi2[ii]) & (d2 > lo2[ii])
        mem_i.append(ii[hit])
        mem_p.append(pts[hit])
    mi = np.concatenate(mem_i)
    mp = np.concatenate(mem_p)
    order = np.lexsort((mp, mi))          # by shell, then meshgrid C-order (== X[circle] order)
    mi, mp = mi[order], mp[order]
    out = np.zeros((mi.size + 1, 4))
    out[1:, 0] = rs[mi]
    out[1:, 1] = X.ravel()[mp]
    out[1:, 2] = Y.ravel()[mp]
    out[1:, 3] = Z.ravel()[mp]
    out.setflags(write=False)
    return out


def sphere_pix(vox, radius=50) -> np.ndarray:
    """The (rows, 4) float64 table of CI.getSpherePix(vox, radius) (CI.py:33-63)."""
    key = tuple(float(v) for v in vox)
    return _sphere_pix_cached(key, int(radius))


def radii_indices(table: np.ndarray) -> np.ndarray:
    """CI.py:79-85: prefix lengths b at which a new radius starts (rows [0, b) = radius <= r[b-1])."""
    return np.where(np.diff(table[:, 0]) > 0)[0] + 1


class SphereTable:
    """Device-ready view of a sphere table for one array shape."""

    def __init__(self, offsets, bounds, radii, dup, key=None):
        self.key = key           # content key (vox, Rmax, R, C) when built by compact_table_for
        self.offsets = offsets   # int16 [rows, 3]  (dx, dy, dz)
        self.bounds = bounds     # int32 [nb]      prefix lengths tested in order (CI.py:94)
        self.radii = radii       # float64 [nb]    r[b-1] for each bound (CI.py:105)
        self.dup = dup           # uint8 [rows]    1 = linear offset already seen in an earlier row

    @property
    def rows(self):
        return int(self.offsets.shape[0])


@functools.lru_cache(maxsize=16)
def _compact_cached(vox_key: tuple, radius: int, shape: tuple) -> SphereTable:
    t = compact_table(_sphere_pix_cached(vox_key, radius), shape)
    t.key = (vox_key, radius, shape[0], shape[1])   # the table depends on (vox, Rmax, R, C) only
    return t


def compact_table_for(vox, radius, shape) -> SphereTable:
    """compact_table(sphere_pix(vox, radius), shape), built once per (vox, radius, shape): the
    same object each call, so its device copy (_lib Context.ci_table) is uploaded once."""
    return _compact_cached(tuple(float(v) for v in vox), int(radius), tuple(int(s) for s in shape))


def compact_table(table: np.ndarray, shape) -> SphereTable:
    s0, s1, _ = (int(s) for s in shape)
    offs = table[:, 1:4].astype(np.int64)
    lin = offs[:, 0] + offs[:, 1] * s0 + offs[:, 2] * s0 * s1
    _, first = np.unique(lin, return_index=True)
    dup = np.ones(lin.size, np.uint8)
    dup[first] = 0
    b = radii_indices(table).astype(np.int32)
    return SphereTable(np.ascontiguousarray(offs.astype(np.int16)), np.ascontiguousarray(b),
                       np.ascontiguousarray(table[b - 1, 0]), dup)
