"""ORACLE -- test infrastructure only.  ctypes access to the C restatements in oracle/*.c
(n4_oracle.c: N4, parity unpinned; ci_oracle.c: cluster index, pinned to CI.py goldens)."""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(HERE, f) for f in ("ci_oracle.c", "n4_oracle.c", "Makefile")]
        if not os.path.exists(LIB) or max(os.path.getmtime(s) for s in srcs) > os.path.getmtime(LIB):
            build()
        _lib = ct.CDLL(LIB)
        _lib.ci_oracle.restype = ct.c_int
        _lib.n4_oracle.restype = ct.c_int
    return _lib


class N4Params(ct.Structure):
    _fields_ = [("n_levels", ct.c_int32), ("max_iters", ct.c_int32 * 8),
                ("conv_threshold", ct.c_float), ("ncp", ct.c_int32 * 3),
                ("spline_order", ct.c_int32), ("n_bins", ct.c_int32),
                ("wiener_noise", ct.c_float), ("fwhm", ct.c_float), ("conv_mode", ct.c_int32)]


def n4_params(max_iters=(50, 50, 50, 50), conv_threshold=0.001, ncp=(4, 4, 4), n_bins=200,
              wiener_noise=0.01, fwhm=0.15, conv_mode=0):
    p = N4Params()
    p.n_levels = len(max_iters)
    for i, m in enumerate(max_iters):
        p.max_iters[i] = m
    p.conv_threshold = conv_threshold
    for i in range(3):
        p.ncp[i] = ncp[i]
    p.spline_order = 3
    p.n_bins = n_bins
    p.wiener_noise = wiener_noise
    p.fwhm = fwhm
    p.conv_mode = conv_mode
    return p


def _ptr(a, t):
    return a.ctypes.data_as(ct.POINTER(t))


def n4(I, mask, **kw):
    """Returns (corrected float32, iterations per level, final convergence per level)."""
    I = np.ascontiguousarray(I, dtype=np.float32)
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    prm = n4_params(**kw)
    out = np.empty_like(I)
    its = np.zeros(prm.n_levels, np.int32)
    conv = np.zeros(prm.n_levels, np.float32)
    rc = lib().n4_oracle(_ptr(I, ct.c_float), _ptr(m, ct.c_uint8), ct.c_int64(I.shape[0]),
                         ct.c_int64(I.shape[1]), ct.c_int64(I.shape[2]), ct.byref(prm),
                         _ptr(out, ct.c_float), _ptr(its, ct.c_int32), _ptr(conv, ct.c_float))
    if rc:
        raise RuntimeError(f"n4_oracle rc={rc}")
    return out, its, conv


def n4_itk(I, mask, nonpos_raw=False, threads=1, spec=0, **kw):
    """n4_oracle.c mode 1: ITK-like float (RealType) arithmetic in raster order, one thread.  Only
    for measuring how far the build spec's precision choices sit from an ITK-like float pipeline
    (DESIGN.md §6); the GPU is never compared with it bit for bit.  spec: bit k takes the build
    spec's form of stage Sk instead (1 log, 3 histogram, 5 fit, 6 evaluation, 7 exp, 9 output)."""
    I = np.ascontiguousarray(I, dtype=np.float32)
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    prm = n4_params(**kw)
    out = np.empty_like(I)
    its = np.zeros(prm.n_levels, np.int32)
    conv = np.zeros(prm.n_levels, np.float32)
    lib().n4_oracle_itk.restype = ct.c_int
    rc = lib().n4_oracle_itk(_ptr(I, ct.c_float), _ptr(m, ct.c_uint8), ct.c_int64(I.shape[0]),
                             ct.c_int64(I.shape[1]), ct.c_int64(I.shape[2]), ct.byref(prm),
                             ct.c_int(1 if nonpos_raw else 0), ct.c_int(threads), ct.c_int(spec),
                             _ptr(out, ct.c_float),
                             _ptr(its, ct.c_int32), _ptr(conv, ct.c_float))
    if rc:
        raise RuntimeError(f"n4_oracle_itk rc={rc}")
    return out, its, conv


def ci(defect, table, vox):
    """Cluster-index map (float64, C-order) and per-voxel shell index (-1 off-defect).
    ``table`` is a vent_analysis_amd.sphere.SphereTable (reference-identical rows)."""
    d = np.ascontiguousarray(np.asarray(defect) != 0, dtype=np.uint8)
    out = np.zeros(d.shape, np.float64)
    shell = np.zeros(d.shape, np.int32)
    rc = lib().ci_oracle(_ptr(d, ct.c_uint8), ct.c_int64(d.shape[0]), ct.c_int64(d.shape[1]),
                         ct.c_int64(d.shape[2]), _ptr(table.offsets, ct.c_int16),
                         _ptr(table.dup, ct.c_uint8), ct.c_int64(table.rows),
                         _ptr(table.bounds, ct.c_int32), _ptr(table.radii, ct.c_double),
                         ct.c_int64(table.bounds.shape[0]), ct.c_double(float(np.min(vox))),
                         _ptr(out, ct.c_double), _ptr(shell, ct.c_int32))
    if rc == 2:
        raise ValueError("cluster index: maximum radius reached (CI.py:101-103)")
    if rc:
        raise RuntimeError(f"ci_oracle rc={rc}")
    return out, shell
