"""ctypes binding of libventhip.so (include/vent_hip.h).

The library is built in-tree (``python __graft_entry__.py`` / ``make -C vent_analysis_amd/csrc``)
and MUST be present: there is no CPU fallback.  Every status code is mapped to the Python
exception the reference raises at the same point (SURVEY.md §8b "Errors").
"""
from __future__ import annotations

import atexit
import ctypes as ct
import os
import threading
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VH_LIB_PATH") or os.path.join(HERE, "libventhip.so")   # override: A/B builds

VH_OK, VH_ERR_ARG, VH_ERR_HIP, VH_ERR_NOMEM, VH_ERR_MAXRADIUS, VH_ERR_EMPTY, VH_ERR_RCCL, \
    VH_ERR_NODEV, VH_ERR_INDEX = range(9)
COHORT_BINS = 1024
COMM_ID_BYTES = 128


class N4Params(ct.Structure):
    _fields_ = [("n_levels", ct.c_int32), ("max_iters", ct.c_int32 * 8),
                ("conv_threshold", ct.c_float), ("ncp", ct.c_int32 * 3),
                ("spline_order", ct.c_int32), ("n_bins", ct.c_int32),
                ("wiener_noise", ct.c_float), ("fwhm", ct.c_float), ("conv_mode", ct.c_int32)]


class VdpResult(ct.Structure):
    _fields_ = [("vdp", ct.c_double), ("vdp_lb", ct.c_double), ("vdp_km", ct.c_double),
                ("defect_volume", ct.c_double), ("lung_volume", ct.c_double),
                ("km_centres", ct.c_double * 4), ("snr", ct.c_double),
                ("mean_anchor", ct.c_float), ("p99", ct.c_float),
                ("n_mask", ct.c_int64), ("n_defect", ct.c_int64), ("n_lb12", ct.c_int64),
                ("n_km0", ct.c_int64), ("n4_iters", ct.c_int32 * 8), ("n4_conv", ct.c_float * 8)]


class RunOpts(ct.Structure):
    _fields_ = [("do_n4", ct.c_int32), ("n4", N4Params), ("thresh", ct.c_float),
                ("do_snr", ct.c_int32), ("do_kmeans", ct.c_int32), ("do_cohort", ct.c_int32),
                ("profile", ct.c_int32), ("vox", ct.c_double * 3), ("n4_subbatch", ct.c_int32),
                ("morph3d", ct.c_int32), ("n4_mode", ct.c_int32)]


class VentHipError(RuntimeError):
    pass


_P = ct.c_void_p
_I64 = ct.c_int64
_SIGS = {
    "vh_abi_version": ([], ct.c_int),
    "vh_status_string": ([ct.c_int], ct.c_char_p),
    "vh_device_count": ([ct.POINTER(ct.c_int)], ct.c_int),
    "vh_n4_default_params": ([ct.POINTER(N4Params)], None),
    "vh_default_run_opts": ([ct.POINTER(RunOpts)], None),
    "vh_create": ([ct.c_int, ct.POINTER(_P)], ct.c_int),
    "vh_destroy": ([_P], ct.c_int),
    "vh_last_error": ([_P], ct.c_char_p),
    "vh_synchronize": ([_P], ct.c_int),
    "vh_n4": ([_P, _P, _P, _I64, _I64, _I64, _I64, ct.POINTER(N4Params), _P, _P, _P], ct.c_int),
    "vh_border": ([_P, _P, _I64, _I64, _I64, _I64, _P], ct.c_int),
    "vh_snr": ([_P, _P, _P, _I64, _I64, _I64, _I64, _P], ct.c_int),
    "vh_vdp": ([_P, _P, _P, _P, _I64, _I64, _I64, _I64, ct.c_float, _P, _P, _P, _P, _P], ct.c_int),
    "vh_ci": ([_P, _P, _I64, _I64, _I64, _I64, _P, _P, _I64, _P, _P, _I64, ct.c_double, _P, _P,
               _P], ct.c_int),
    "vh_ci_table_create": ([_P, _I64, _I64, _P, _P, _I64, _P, _P, _I64, ct.POINTER(_P)], ct.c_int),
    "vh_ci_table_destroy": ([_P], ct.c_int),
    "vh_ci_tab": ([_P, _P, _I64, _I64, _I64, _I64, _P, ct.c_double, _P, _P, _P], ct.c_int),
    "vh_batch_create": ([_P, _I64, _I64, _I64, _I64, ct.POINTER(_P)], ct.c_int),
    "vh_batch_destroy": ([_P], ct.c_int),
    "vh_batch_upload": ([_P, _P, _P], ct.c_int),
    "vh_batch_run": ([_P, ct.POINTER(RunOpts)], ct.c_int),
    "vh_batch_sync": ([_P], ct.c_int),
    "vh_batch_download": ([_P, _P, _P, _P, _P, _P], ct.c_int),
    "vh_batch_cohort_hist": ([_P, _P], ct.c_int),
    "vh_batch_kernel_names": ([], ct.c_char_p),
    "vh_batch_reset_timers": ([_P], ct.c_int),
    "vh_batch_kernel_time": ([_P, ct.c_char_p, ct.POINTER(ct.c_double), ct.POINTER(ct.c_int64),
                              ct.POINTER(ct.c_double)], ct.c_int),
    "vh_batch_study_times": ([_P, _P], ct.c_int),
    "vh_ctx_profile": ([_P, ct.c_int], ct.c_int),
    "vh_ctx_kernel_time": ([_P, ct.c_char_p, ct.POINTER(ct.c_double), ct.POINTER(ct.c_int64)],
                           ct.c_int),
    "vh_overlay": ([_P, _P, _P, _I64, _I64, _I64, _I64, _P], ct.c_int),
    "vh_montage": ([_P, _I64, _I64, _I64, _P, ct.c_int, _P, ct.c_int, _P, _P, _P, _P, _P, _I64, _P,
                    _P], ct.c_int),
    "vh_recon": ([_P, _P, _I64, _I64, _I64, _P], ct.c_int),
    "vh_pipe_create": ([_P, _I64, _I64, _I64, _I64, ct.c_int, ct.POINTER(_P)], ct.c_int),
    "vh_pipe_run": ([_P, _P, _P, _I64, ct.POINTER(RunOpts), _P, _P, _P, _P, _P], ct.c_int),
    "vh_pipe_destroy": ([_P], ct.c_int),
    "vh_pipe_stats": ([_P, ct.POINTER(ct.c_int64), ct.POINTER(ct.c_int64)], ct.c_int),
    "vh_link_probe": ([_P, ct.c_int64, ct.POINTER(ct.c_double)], ct.c_int),
    "vh_host_alloc": ([_P, ct.c_int64, ct.POINTER(_P)], ct.c_int),
    "vh_host_free": ([_P], ct.c_int),
    "vh_comm_unique_id": ([_P], ct.c_int),
    "vh_comm_init": ([_P, ct.c_int, ct.c_int, _P], ct.c_int),
    "vh_batch_cohort_allreduce": ([_P], ct.c_int),
    "vh_comm_info": ([_P, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int)], ct.c_int),
    "vh_comm_destroy": ([_P], ct.c_int),
}
EXPORTED = tuple(_SIGS)
ABI_VERSION = 8   # include/vent_hip.h VH_ABI_VERSION

_lib = None
_lock = threading.RLock()


def lib():
    """Load libventhip.so; fails loudly when the HIP extension has not been built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"{LIB_PATH} is missing: build it with "
                                      "`python __graft_entry__.py build` (no CPU fallback exists)")
                L = ct.CDLL(LIB_PATH)
                for name, (args, res) in _SIGS.items():
                    f = getattr(L, name)
                    f.argtypes = args
                    f.restype = res
                v = L.vh_abi_version()
                if v != ABI_VERSION:   # a stale build: its structs and signatures differ
                    raise ImportError(f"{LIB_PATH} has ABI version {v}, this shim needs "
                                      f"{ABI_VERSION}: rebuild it (`python __graft_entry__.py build`)")
                _lib = L
    return _lib


def empty_aligned(shape, dtype, align=4096):
    """np.empty whose data starts on a page boundary.  vh_pipe DMAs caller arrays in place, chunk
    by chunk; when every chunk boundary is page aligned (a study is 384 pages at 128x128x24 float32)
    no chunk needs the sub-page head / tail copies through staging, which run as blit kernels that
    wait for a free CU behind the N4 kernel."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    buf = np.empty(n + align, np.uint8)
    off = (-buf.ctypes.data) % align
    return buf[off:off + n].view(dtype).reshape(shape)


def _ptr(a):
    return None if a is None else ct.c_void_p(a.ctypes.data)


class _PinnedPool:
    """Page-locked host buffers (vh_host_alloc) for the arrays an entry point returns: their D2H
    runs at the link rate with no runtime staging.  A returned array's buffer goes back to the pool
    when the last view of it is gone (a finalizer on the ctypes buffer numpy holds as its base); the
    pool keeps at most ``keep`` idle buffers per size.  r4: the CI line's dense f64 map."""

    def __init__(self, ctx, keep=4):
        self.ctx = ctx
        self.keep = keep
        self.idle = {}
        self.lock = threading.Lock()

    def array(self, shape, dtype):
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        with self.lock:
            ptrs = self.idle.get(n)
            ptr = ptrs.pop() if ptrs else None
        if ptr is None:
            h = _P()
            self.ctx.check(self.ctx.L.vh_host_alloc(self.ctx.h, n, ct.byref(h)), "vh_host_alloc")
            ptr = h.value
        buf = (ct.c_char * n).from_address(ptr)
        weakref.finalize(buf, self._release, n, ptr)
        return np.frombuffer(buf, dtype).reshape(shape)

    def _release(self, n, ptr):
        with self.lock:
            ptrs = self.idle.setdefault(n, [])
            if self.ctx.h is not None and len(ptrs) < self.keep:
                ptrs.append(ptr)
                return
        lib().vh_host_free(ct.c_void_p(ptr))

    def close(self):
        with self.lock:
            for ptrs in self.idle.values():
                for p in ptrs:
                    lib().vh_host_free(ct.c_void_p(p))
            self.idle.clear()


class Context:
    """One device + one HIP stream (vh_ctx)."""

    def __init__(self, device: int = 0):
        self.L = lib()
        h = _P()
        rc = self.L.vh_create(int(device), ct.byref(h))
        if rc != VH_OK:
            raise VentHipError(f"vh_create(device={device}) failed: "
                               f"{self.L.vh_status_string(rc).decode()}")
        self.h = h
        self.device = device
        # (table key, R, C) -> (table, vh_ci_table handle), least recently used first: tables stay
        # in HBM.  ci_lock covers the lookup, any eviction and the vh_ci_tab call that uses the
        # handle, so no thread's handle is destroyed under it
        self.ci_tables = {}
        self.ci_lock = threading.RLock()
        self.pinned = _PinnedPool(self)

    def link_probe(self, nbytes=256 << 20):
        """PCIe rates of this context's GPU with pinned host memory, GB/s: H2D alone, D2H alone,
        both at once on two streams (vh_link_probe)."""
        out = (ct.c_double * 3)()
        self.check(self.L.vh_link_probe(self.h, int(nbytes), out), "vh_link_probe")
        return {"h2d_GBps": round(out[0], 2), "d2h_GBps": round(out[1], 2), "both_GBps": round(out[2], 2)}

    CI_TABLES_KEPT = 16

    def ci_table(self, table, R, C):
        """The device copy of a compact sphere table for (R, C) volumes (vh_ci_table_create, once
        per table content; the reference caches the table file the same way, CI.py:43-61).  Keyed
        by ``table.key`` -- (vox, Rmax, R, C) for sphere.compact_table_for's tables -- or by the
        object for ad-hoc tables.  Call with ``ci_lock`` held for as long as the handle is used."""
        tk = getattr(table, "key", None)
        key = (tk if tk is not None else ("obj", id(table)), int(R), int(C))
        hit = self.ci_tables.pop(key, None)
        if hit is not None and (tk is not None or hit[0] is table):
            self.ci_tables[key] = hit   # most recently used last
            return hit[1]
        if hit is not None:   # an ad-hoc table whose id was reused
            self.L.vh_ci_table_destroy(hit[1])
        while len(self.ci_tables) >= self.CI_TABLES_KEPT:   # drop the least recently used
            k0 = next(iter(self.ci_tables))
            self.L.vh_ci_table_destroy(self.ci_tables.pop(k0)[1])   # locks ctx->mu, drains
        h = _P()
        self.check(self.L.vh_ci_table_create(self.h, int(R), int(C), _ptr(table.offsets),
                                             _ptr(table.dup), table.rows, _ptr(table.bounds),
                                             _ptr(table.radii), table.bounds.shape[0], ct.byref(h)),
                   "vh_ci_table_create")
        self.ci_tables[key] = (table, h)
        return h

    def close(self):
        if getattr(self, "h", None):
            self.pinned.close()
            with self.ci_lock:
                for _, th in self.ci_tables.values():
                    self.L.vh_ci_table_destroy(th)
                self.ci_tables.clear()
            self.L.vh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, where: str):
        if rc == VH_OK:
            return
        msg = (self.L.vh_last_error(self.h) or b"").decode() if self.h else ""
        text = f"{where}: {self.L.vh_status_string(rc).decode()}: {msg}"
        if rc == VH_ERR_MAXRADIUS:
            raise ValueError(text)
        if rc in (VH_ERR_EMPTY, VH_ERR_INDEX):
            raise IndexError(text)
        if rc == VH_ERR_ARG:
            raise ValueError(text)
        if rc == VH_ERR_NOMEM:
            raise MemoryError(text)
        raise VentHipError(text)


_ctx = {}
_live = weakref.WeakSet()   # open Batch / Pipe objects


@atexit.register
def _shutdown():
    """Destroy the cached contexts (their scratch batches, streams and device buffers) while the HIP
    runtime -- and a profiler attached to it -- is still fully up.  Left to interpreter teardown,
    vh_destroy ran in no defined order, possibly after C-level exit handlers had started taking the
    runtime and rocprofv3 down (SIGSEGV in exit() after profiled cooperative launches)."""
    with _lock:
        _batch_pool.clear()
        for o in list(_live):   # batches and pipes first: they hold their context
            try:
                o.close()
            except Exception:
                pass
        for c in list(_ctx.values()):
            try:
                c.close()
            except Exception:
                pass
        _ctx.clear()


def context(device: int = 0) -> Context:
    c = _ctx.get(device)
    if c is None:
        with _lock:
            c = _ctx.get(device)
            if c is None:
                c = Context(device)
                _ctx[device] = c
    return c


def device_count() -> int:
    n = ct.c_int(0)
    lib().vh_device_count(ct.byref(n))
    return n.value


def n4_params(max_iters=(50, 50, 50, 50), conv_threshold=0.001, ncp=(4, 4, 4), n_bins=200,
              wiener_noise=0.01, fwhm=0.15, conv_mode=0) -> N4Params:
    """SimpleITK N4BiasFieldCorrectionImageFilter defaults (Vent_Analysis.py:330).  conv_mode 0 is
    ITK's float Welford convergence measure (reference iteration counts); 1 the exact CoV."""
    p = N4Params()
    lib().vh_n4_default_params(ct.byref(p))
    p.n_levels = len(max_iters)
    for i in range(8):
        p.max_iters[i] = max_iters[i] if i < len(max_iters) else 0
    p.conv_threshold = conv_threshold
    for i in range(3):
        p.ncp[i] = ncp[i]
    p.n_bins = n_bins
    p.wiener_noise = wiener_noise
    p.fwhm = fwhm
    p.conv_mode = int(conv_mode)
    return p


def as_batch(a, dtype):
    """(R,C,Z) or (B,R,C,Z) -> contiguous (B,R,C,Z) of dtype (DICOM arrays are transposed views,
    Vent_Analysis.py:179, so a contiguous copy is made when needed)."""
    a = np.asarray(a)
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4:
        raise ValueError(f"expected a 3-D volume or a 4-D batch, got shape {a.shape}")
    return np.ascontiguousarray(a, dtype=dtype)


# ---- thin wrappers over the host-buffer entry points -------------------------------------------
def n4(hp, mask, device=0, **kw):
    c = context(device)
    h = as_batch(hp, np.float32)
    m = as_batch(mask, np.uint8)
    if h.shape != m.shape:
        raise ValueError("HPvent and mask shapes differ")
    B, R, C, Z = h.shape
    p = n4_params(**kw)
    out = np.empty_like(h)
    its = np.zeros((B, p.n_levels), np.int32)
    conv = np.zeros((B, p.n_levels), np.float32)
    c.check(c.L.vh_n4(c.h, _ptr(h), _ptr(m), R, C, Z, B, ct.byref(p), _ptr(out), _ptr(its),
                      _ptr(conv)), "vh_n4")
    return out, its, conv


def border(a, device=0):
    c = context(device)
    x = as_batch(a, np.uint8)
    B, R, C, Z = x.shape
    out = np.empty_like(x)
    c.check(c.L.vh_border(c.h, _ptr(x), R, C, Z, B, _ptr(out)), "vh_border")
    return out


def snr(hp, mask, device=0):
    c = context(device)
    h = as_batch(hp, np.float32)
    m = as_batch(mask, np.uint8)
    B, R, C, Z = h.shape
    out = np.zeros(B, np.float64)
    c.check(c.L.vh_snr(c.h, _ptr(h), _ptr(m), R, C, Z, B, _ptr(out)), "vh_snr")
    return out


def vdp(n4v, mask, vox, hp=None, thresh=0.6, device=0):
    c = context(device)
    n = as_batch(n4v, np.float32)
    m = as_batch(mask, np.uint8)
    h = None if hp is None else as_batch(hp, np.float32)
    B, R, C, Z = n.shape
    defect = np.empty((B, R, C, Z), np.uint8)
    bord = np.empty_like(defect)
    lb = np.empty_like(defect)
    res = (VdpResult * B)()
    vx = np.ascontiguousarray(vox, dtype=np.float64)
    c.check(c.L.vh_vdp(c.h, _ptr(h), _ptr(n), _ptr(m), R, C, Z, B, ct.c_float(thresh), _ptr(vx),
                       _ptr(defect), _ptr(bord), _ptr(lb), ct.cast(res, ct.c_void_p)), "vh_vdp")
    return defect, bord, lb, list(res)


def ci(defect, table, minvox, device=0, shell=True, out=None):
    """table: vent_analysis_amd.sphere.SphereTable for this shape (kept in HBM per context after
    the first call).  Returns (ci f64, scalar[B], shell int32 or None).  The map goes into a pooled
    page-locked buffer the scatter kernel writes directly (vh_host_alloc), or into ``out`` (a
    C-contiguous f64 array of the batch's shape: then through a device map and one copy)."""
    c = context(device)
    d = np.asarray(defect)
    if d.dtype == np.bool_:
        d = d.view(np.uint8)   # (no copy: the kernels test != 0)
    elif d.dtype != np.uint8:
        d = d != 0
    d = as_batch(d, np.uint8)   # a u8 map goes in as it is (nonzero = defect, CI.py:37)
    B, R, C, Z = d.shape
    if out is None:
        out = c.pinned.array((B, R, C, Z), np.float64)   # page-locked, device-mapped: no copy
    elif out.dtype != np.float64 or out.size != B * R * C * Z or not out.flags.c_contiguous:
        raise ValueError("ci: out must be a C-contiguous float64 array of the batch's size")
    sh = np.empty((B, R, C, Z), np.int32) if shell else None
    sc = np.zeros(B, np.float64)
    with c.ci_lock:
        th = c.ci_table(table, R, C)
        c.check(c.L.vh_ci_tab(c.h, _ptr(d), R, C, Z, B, th, ct.c_double(minvox), _ptr(out), _ptr(sc),
                              _ptr(sh)), "vh_ci_tab")
    return out, sc, sh


def ctx_profile(on, device=0):
    """Time the kernel classes of the host-buffer entry points (vh_ci, ...) on this device's
    context (vh_ctx_profile); switching discards earlier timings."""
    c = context(device)
    c.check(c.L.vh_ctx_profile(c.h, 1 if on else 0), "vh_ctx_profile")


def ctx_kernel_time(name, device=0):
    """(total ms, launches) of a kernel class timed since ctx_profile(True)."""
    c = context(device)
    ms, n = ct.c_double(), ct.c_int64()
    c.check(c.L.vh_ctx_kernel_time(c.h, name.encode(), ct.byref(ms), ct.byref(n)), "vh_ctx_kernel_time")
    return ms.value, n.value


def overlay(n4, defect, device=0):
    """exportDICOM pixel data (vh_overlay): uint8 [B][Z][R][C][3] for (B, R, C, Z) inputs (a
    single volume gives [Z][R][C][3])."""
    c = context(device)
    single = np.ndim(n4) == 3
    n = as_batch(n4, np.float32)
    d = as_batch(defect, np.uint8) if np.asarray(defect).dtype == np.uint8 else \
        as_batch(np.where(np.asarray(defect) == 1, 1, np.where(np.asarray(defect) == 0, 0, 2)), np.uint8)
    B, R, C, Z = n.shape
    out = np.empty((B, Z, R, C, 3), np.uint8)
    c.check(c.L.vh_overlay(c.h, _ptr(n), _ptr(d), R, C, Z, B, _ptr(out)), "vh_overlay")
    return out[0] if single else out


def montage(proton, hp, n4, mask_border, defect, ci, parula, crop, device=0):
    """screenShot's montage array (vh_montage): uint8 [7 nr][ns nc][3].  crop = (r0, nr, c0, nc,
    s0, ns); ci None = the blank CI panel."""
    c = context(device)

    def fl(a):
        a = np.asarray(a)
        if a.dtype == np.float64:
            return np.ascontiguousarray(a), 1
        return np.ascontiguousarray(a, dtype=np.float32), 0
    p, p64 = fl(proton)
    h, h64 = fl(hp)
    n = np.ascontiguousarray(n4, dtype=np.float32)
    R, C, Z = n.shape
    mb = np.ascontiguousarray(np.asarray(mask_border) != 0, dtype=np.uint8)
    df = np.ascontiguousarray(np.asarray(defect) != 0, dtype=np.uint8)
    ci64 = None if ci is None else np.ascontiguousarray(ci, dtype=np.float64)
    pal = np.ascontiguousarray(parula, dtype=np.float64)
    cr = np.ascontiguousarray(crop, dtype=np.int64)
    img = np.empty((7 * int(cr[1]), int(cr[5]) * int(cr[3]), 3), np.uint8)
    c.check(c.L.vh_montage(c.h, R, C, Z, _ptr(p), p64, _ptr(h), h64, _ptr(n), _ptr(mb), _ptr(df),
                           _ptr(ci64), _ptr(pal), pal.shape[0], _ptr(cr), _ptr(img)), "vh_montage")
    return img


def recon(raw_k, device=0):
    """process_RAW's image (vh_recon, Vent_Analysis.py:537-540): complex k-space [n0][n1][nz] ->
    complex128 [n1][n0][nz] = transpose(fftshift(fft2(fftshift(slice))), (1, 0, 2))[:, ::-1, :].
    The transform runs in complex128 whatever the input precision (numpy 1.23, the reference pin,
    computes every FFT in double)."""
    c = context(device)
    k = np.asarray(raw_k)
    if k.ndim != 3:
        raise ValueError(f"raw k-space must be 3-D (cols, lines, slices), got shape {k.shape}")
    k = np.ascontiguousarray(k, dtype=np.complex128)
    n0, n1, nz = k.shape
    out = np.empty((n1, n0, nz), np.complex128)
    c.check(c.L.vh_recon(c.h, _ptr(k), n0, n1, nz, _ptr(out)), "vh_recon")
    return out


class Batch:
    """Device-resident batch of studies (vh_batch): upload once, run the whole pipeline on the
    GPU, download results.  Used by bench.py and for cohort processing."""

    def __init__(self, R, C, Z, n, device=0):
        self.ctx = context(device)
        self.L = self.ctx.L
        self.shape = (int(n), int(R), int(C), int(Z))
        h = _P()
        self.ctx.check(self.L.vh_batch_create(self.ctx.h, R, C, Z, n, ct.byref(h)),
                       "vh_batch_create")
        self.h = h
        _live.add(self)

    def close(self):
        if getattr(self, "h", None):
            self.L.vh_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, hp, mask):
        h = np.ascontiguousarray(hp, dtype=np.float32)
        m = np.ascontiguousarray(mask, dtype=np.uint8)
        if h.shape != self.shape or m.shape != self.shape:
            raise ValueError(f"batch expects {self.shape}")
        self.ctx.check(self.L.vh_batch_upload(self.h, _ptr(h), _ptr(m)), "vh_batch_upload")

    @staticmethod
    def options(do_n4=True, thresh=0.6, do_snr=True, do_kmeans=True, do_cohort=False,
                profile=False, vox=(1.0, 1.0, 1.0), n4_subbatch=0, morph3d=False,
                n4_mode=0, **n4kw) -> RunOpts:
        o = RunOpts()
        lib().vh_default_run_opts(ct.byref(o))
        o.do_n4 = int(bool(do_n4))
        o.n4 = n4_params(**n4kw)
        o.thresh = thresh
        o.do_snr = int(bool(do_snr))
        o.do_kmeans = int(bool(do_kmeans))
        o.do_cohort = int(bool(do_cohort))
        o.profile = int(bool(profile))
        for i in range(3):
            o.vox[i] = float(vox[i])
        o.n4_subbatch = int(n4_subbatch)
        o.morph3d = int(bool(morph3d))
        o.n4_mode = {"auto": 0, "sweep": 1, "study": 2, "grid": 3}.get(n4_mode, n4_mode)
        return o

    def run(self, opts: RunOpts):
        self.ctx.check(self.L.vh_batch_run(self.h, ct.byref(opts)), "vh_batch_run")

    def sync(self):
        self.ctx.check(self.L.vh_batch_sync(self.h), "vh_batch_sync")

    def download(self, n4=False, maps=True):
        B = self.shape[0]
        out_n4 = np.empty(self.shape, np.float32) if n4 else None
        d = np.empty(self.shape, np.uint8) if maps else None
        bo = np.empty(self.shape, np.uint8) if maps else None
        lb = np.empty(self.shape, np.uint8) if maps else None
        res = (VdpResult * B)()
        self.ctx.check(self.L.vh_batch_download(self.h, _ptr(out_n4), _ptr(d), _ptr(bo), _ptr(lb),
                                                ct.cast(res, ct.c_void_p)), "vh_batch_download")
        return out_n4, d, bo, lb, list(res)

    def cohort_hist(self):
        h = np.zeros(COHORT_BINS, np.uint64)
        self.ctx.check(self.L.vh_batch_cohort_hist(self.h, _ptr(h)), "vh_batch_cohort_hist")
        return h

    def cohort_allreduce(self):
        self.ctx.check(self.L.vh_batch_cohort_allreduce(self.h), "vh_batch_cohort_allreduce")

    def reset_timers(self):
        self.ctx.check(self.L.vh_batch_reset_timers(self.h), "vh_batch_reset_timers")

    def study_times(self):
        """Per-study wall time (us) of the last run's one-workgroup-per-study N4 kernel."""
        us = np.zeros(self.shape[0], np.float64)
        self.ctx.check(self.L.vh_batch_study_times(self.h, _ptr(us)), "vh_batch_study_times")
        return us

    def kernel_time(self, name):
        ms, n, by = ct.c_double(0), ct.c_int64(0), ct.c_double(0)
        self.ctx.check(self.L.vh_batch_kernel_time(self.h, name.encode(), ct.byref(ms),
                                                   ct.byref(n), ct.byref(by)),
                       "vh_batch_kernel_time")
        return ms.value, n.value, by.value


_batch_pool = {}   # (device, R, C, Z, n) -> idle Batch objects (pooled_batch)
_BATCH_POOL_KEEP = 2


class pooled_batch:
    """A device-resident batch of this shape for the length of a ``with`` block, reused across calls
    (the class's one-study calculate_VDP: creating a batch allocates its device workspace, which cost
    more than the pipeline itself on a 128x128x24 study).  Exclusive while held, so host threads never
    share one; at most _BATCH_POOL_KEEP idle batches per shape stay allocated (the rest are closed)."""

    def __init__(self, R, C, Z, n=1, device=0):
        self.key = (int(device), int(R), int(C), int(Z), int(n))

    def __enter__(self):
        with _lock:
            idle = _batch_pool.get(self.key)
            self.b = idle.pop() if idle else None
        if self.b is None or self.b.h is None:
            self.b = Batch(*self.key[1:], device=self.key[0])
        return self.b

    def __exit__(self, exc_type, exc, tb):
        b = self.b
        if exc_type is not None:   # a failed call may have left the batch in any state
            b.close()
            return False
        with _lock:
            idle = _batch_pool.setdefault(self.key, [])
            if len(idle) < _BATCH_POOL_KEEP:
                idle.append(b)
                return False
        b.close()
        return False


class Pipe:
    """Host-to-host pipeline (vh_pipe): n host-resident studies streamed through `slots` device
    batches of `sub` volumes, transfers of one sub-batch overlapping the compute of another."""

    def __init__(self, R, C, Z, sub, slots=3, device=0):
        self.ctx = context(device)
        self.L = self.ctx.L
        self.vshape = (int(R), int(C), int(Z))
        h = _P()
        self.ctx.check(self.L.vh_pipe_create(self.ctx.h, R, C, Z, sub, slots, ct.byref(h)),
                       "vh_pipe_create")
        self.h = h
        _live.add(self)

    def close(self):
        if getattr(self, "h", None):
            self.L.vh_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, hp, mask, opts: RunOpts, n4=True, maps=True, out=None):
        """Returns (n4, defect, border, lb, results) host arrays for all len(hp) studies; `out`
        may pass preallocated (n4, defect, border, lb) arrays."""
        h = np.ascontiguousarray(hp, dtype=np.float32)
        m = np.ascontiguousarray(mask, dtype=np.uint8)
        n = h.shape[0]
        if h.shape[1:] != self.vshape or m.shape != h.shape:
            raise ValueError(f"pipe expects (n,) + {self.vshape}")
        if out is None:
            out = (empty_aligned(h.shape, np.float32) if n4 else None,
                   empty_aligned(h.shape, np.uint8) if maps else None,
                   empty_aligned(h.shape, np.uint8) if maps else None,
                   empty_aligned(h.shape, np.uint8) if maps else None)
        res = (VdpResult * n)()
        self.ctx.check(self.L.vh_pipe_run(self.h, _ptr(h), _ptr(m), n, ct.byref(opts),
                                          *[_ptr(a) for a in out], ct.cast(res, ct.c_void_p)),
                       "vh_pipe_run")
        return (*out, list(res))

    def stats(self):
        """(peak bytes of caller memory pinned in place, caller ranges staged instead) of the last
        run (vh_pipe_stats)."""
        pk, st = ct.c_int64(), ct.c_int64()
        self.ctx.check(self.L.vh_pipe_stats(self.h, ct.byref(pk), ct.byref(st)), "vh_pipe_stats")
        return int(pk.value), int(st.value)


def comm_unique_id() -> bytes:
    buf = np.zeros(COMM_ID_BYTES, np.uint8)
    rc = lib().vh_comm_unique_id(_ptr(buf))
    if rc != VH_OK:
        raise VentHipError("ncclGetUniqueId failed")
    return buf.tobytes()


def comm_init(nranks: int, rank: int, uid: bytes, device=0):
    c = context(device)
    buf = np.frombuffer(uid, np.uint8).copy()
    c.check(c.L.vh_comm_init(c.h, nranks, rank, _ptr(buf)), "vh_comm_init")


def comm_info(device=0):
    """(ranks, rank) of the context's RCCL communicator as RCCL reports them (vh_comm_info)."""
    c = context(device)
    n, r = ct.c_int(0), ct.c_int(-1)
    c.check(c.L.vh_comm_info(c.h, ct.byref(n), ct.byref(r)), "vh_comm_info")
    return n.value, r.value


def comm_destroy(device=0):
    """Releases the context's RCCL communicator (vh_comm_destroy)."""
    c = context(device)
    c.L.vh_comm_destroy(c.h)
