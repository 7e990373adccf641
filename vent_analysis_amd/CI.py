"""Cluster index -- drop-in for the reference's CI module (CI.py:1-145), computed on the GPU.

Same function names and argument meaning as CI.py.  ``calculate_CI`` runs the sphere-growing
cluster value of every defect voxel in one HIP kernel (vent_analysis_amd/csrc/ci.hip); the small
index helpers keep the reference's exact (MATLAB-style) semantics because callers may rely on
them.  No CPU fallback: without libventhip.so the import of the GPU path fails loudly.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .sphere import compact_table, compact_table_for, radii_indices, sphere_pix

__all__ = ["multi_which", "getSpherePix", "px2vec", "vec2px", "getRadiiIndices", "calculate_CV",
           "calculate_CI", "calculate_CI_with_index"]


def multi_which(A):
    """All row/col/slice indices of the ones of A, C order (CI.py:10-30)."""
    if np.isscalar(A):
        return np.where(A)[0]
    return np.argwhere(np.asarray(A).ravel().reshape(np.shape(A)) != 0).astype(int)


def getSpherePix(vox, radius):
    """(rows, 4) float64 [r, dx, dy, dz] sphere-growing table (CI.py:33-63).  Identical rows to the
    reference's cached '{v0}x{v1}x{v2}_{R}.npy' (checked bit-for-bit in the tests); built in memory
    instead of the cwd file cache."""
    return np.array(sphere_pix(vox, radius))


def px2vec(i, j, k, arrayShape):
    """CI.py:65-68: i + (j-1) s0 + (k-1) s0 s1 with 0-based i, j, k (MATLAB-style offset kept)."""
    return i + (j - 1) * arrayShape[0] + (k - 1) * arrayShape[0] * arrayShape[1]


def vec2px(n, arrayShape):
    """CI.py:70-77 (unused by the reference pipeline; kept for API parity)."""
    s = np.ceil(n / (arrayShape[0] * arrayShape[1]))
    n = n - (s - 1) * arrayShape[1] * arrayShape[0]
    c = np.ceil(n / arrayShape[0])
    r = n - (c - 1) * arrayShape[0]
    return int(r), int(c), int(s)


def getRadiiIndices(data):
    """CI.py:79-85: prefix lengths at which a new radius starts."""
    return radii_indices(np.asarray(data))


def calculate_CI_with_index(defectArray, vox=(1, 1, 1), Rmax=50, device=0):
    """GPU cluster-index map plus the 95th-percentile CI of Vent_Analysis.calculate_CI
    (Vent_Analysis.py:268-270), from one kernel pass.  Returns (CIarray float64, CI float64)."""
    d = np.asarray(defectArray)
    table = compact_table_for(vox, Rmax, d.shape)
    ci, scal, _ = _lib.ci(d, table, float(np.min(vox)), device=device, shell=False)
    # the map is kept for the object's life (Vent_Analysis.CIarray): copied out of the pooled
    # page-locked buffer, which then goes back to the pool (no pinned memory per study)
    return np.array(ci[0]), np.float64(scal[0])


def calculate_CI(defectArray, vox=[1, 1, 1], Rmax=50, type='fast'):   # noqa: A002 (reference name)
    """CI.py:107-145.  Cluster value r * min(vox) at every defect voxel, 0 elsewhere (float64).
    ``type`` ('fast' / 'slow') selected two CPU schedules in the reference; both give the same
    map, which the GPU computes in one pass.  Raises ValueError when a sphere reaches the table's
    maximum radius (CI.py:101-103) and IndexError for an empty defect map."""
    if type not in ("fast", "slow"):
        return None   # the reference falls through both branches and hits an unbound CI
    return calculate_CI_with_index(defectArray, vox, Rmax)[0]


def calculate_CV(defectArrayShape, activeVoxel, defVec, spherePx):
    """CI.py:87-105: [i, j, k, r] for one defect voxel.  Rebuilds the defect map from defVec
    (px2vec indices) and evaluates it with the GPU kernel."""
    s0, s1, s2 = (int(v) for v in defectArrayShape)
    L = np.asarray(defVec, dtype=np.int64) + s0 + s0 * s1   # undo the (j-1), (k-1) offsets
    d = np.zeros((s0, s1, s2), np.uint8)
    a = L % s0
    b = (L // s0) % s1
    c = L // (s0 * s1)
    d[a, b, c] = 1
    spherePx = np.asarray(spherePx)
    table = compact_table(spherePx, d.shape)
    # minvox = 1 gives the raw radius r[b-1]
    ci, _, _ = _lib.ci(d, table, 1.0)
    i, j, k = (int(v) for v in activeVoxel)
    return np.append(np.asarray(activeVoxel), ci[0][i, j, k])
