"""Test-only stand-in for vent_analysis_amd._lib (the ctypes shim of libventhip.so), for driving
bench.main() itself on the CPU: ``bench.py --dry-run`` loads this module in place of the library
(bench.load_lib), so the N > 1 line's host code -- the communicator rank check, the cohort
all-reduce and its check_cohort self-check, max-over-ranks timing, per-rank rates, the isolated
runs, the roofline block, the host-to-host leg under the per-rank pin budget -- runs as it does on
the GPU boxes.  Nothing here is measured or shipped.

Only the surface bench.main() calls is provided.  Each "step" computes the per-rank cohort
histogram rows with numpy (the semantics of k_cohort_search / k_cohort_sum: 1024 bins of the
p99-normalised masked values in [0, 1.5)), and the stand-in communicator's all-reduce is a gloo
all-reduce of those rows (RCCL's ncclAllReduce on the GPU).  Fault injection for the tests:
  VH_DRY_FAIL_RANK=r   rank r exits with status 3 while setting up its communicator
  VH_DRY_BAD_SUM=r     rank r's stand-in all-reduce returns the sum + 1 (a wrong collective)
  VH_DRY_BAD_RANKS=r   rank r's communicator reports one rank too many (vh_comm_info)
"""
from __future__ import annotations

import os
import time
import types

import numpy as np

from vent_analysis_amd._lib import COHORT_BINS, COMM_ID_BYTES, empty_aligned  # noqa: F401

LIB_PATH = None          # no shared object: bench.lib_digest() gives None, no PMC summary matches
COMM_KIND = "gloo stand-in (tests/standin_lib.py, --dry-run)"
PIN_NODE_BUDGET = 32 << 30   # vh_pipe's default page-locking budget per node (api.hip)

# synthetic kernel-class timings per run (ms per launch, launches per run): a multi-launch class
# whose time per step exceeds that of the class with the longest single launch, so the line's
# dominant class shows which rule picked it (time per step: n4_pcg, not sort)
KERNELS = {"n4_pcg": (1.0, 10), "sort": (5.0, 1), "classify": (0.5, 1)}
N4_ITERS = (10, 5, 3, 2)


def _rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_initialized() else 0


def _env_rank(name):
    v = os.environ.get(name)
    return v is not None and v == str(_rank())


def cohort_rows(hp, mk):
    """Per-rank cohort rows (the numpy form of k_cohort_*): 1024 bins over [0, 1.5) of each
    study's masked values divided by its 99th percentile, summed over the batch."""
    h = np.zeros(COHORT_BINS, np.int64)
    for x, m in zip(hp, mk):
        s = np.sort(x[m > 0])
        nv = (x / np.float32(s[int(len(s) * 0.99)])).astype(np.float32)[m > 0]
        nv = nv[(nv >= 0) & (nv < np.float32(1.5))]
        h += np.bincount(np.minimum((nv * np.float32(COHORT_BINS / 1.5)).astype(np.int64),
                                    COHORT_BINS - 1), minlength=COHORT_BINS)
    return h


class _Names:
    @staticmethod
    def vh_batch_kernel_names():
        return ";".join(KERNELS).encode()


def lib():
    return _Names()


class _Ctx:
    def link_probe(self, nbytes=256 << 20):
        return {"h2d_GBps": 50.0, "d2h_GBps": 50.0, "both_GBps": 80.0}


def context(device=0):
    return _Ctx()


class _Result:
    def __init__(self):
        self.n4_iters = list(N4_ITERS) + [0] * 4


_comm = {}


def comm_unique_id():
    return bytes(range(COMM_ID_BYTES))


def comm_init(nranks, rank, uid, device=0):
    if _env_rank("VH_DRY_FAIL_RANK"):
        raise SystemExit(3)
    if len(uid) != COMM_ID_BYTES or uid != comm_unique_id():
        raise RuntimeError("stand-in comm_init: the unique id did not arrive intact")
    _comm.update(nranks=int(nranks), rank=int(rank))


def comm_info(device=0):
    n = _comm["nranks"] + (1 if _env_rank("VH_DRY_BAD_RANKS") else 0)
    return n, _comm["rank"]


def comm_destroy(device=0):
    _comm.clear()


class Batch:
    def __init__(self, R, C, Z, n, device=0):
        self.shape = (int(n), int(R), int(C), int(Z))
        self.hist = np.zeros(COHORT_BINS, np.int64)
        self.reset_timers()

    @staticmethod
    def options(**kw):
        return types.SimpleNamespace(**kw)

    def upload(self, hp, mask):
        if hp.shape != self.shape or mask.shape != self.shape:
            raise ValueError(f"batch expects {self.shape}")
        self.hp, self.mk = hp, mask

    def run(self, opts):
        self.hist = cohort_rows(self.hp, self.mk)
        if getattr(opts, "profile", False):
            for k, (ms, n) in KERNELS.items():
                t = self.timers[k]
                self.timers[k] = (t[0] + ms * n, t[1] + n)

    def cohort_allreduce(self):
        import torch
        import torch.distributed as dist
        if "nranks" not in _comm:
            raise RuntimeError("stand-in: cohort_allreduce before comm_init")
        t = torch.from_numpy(self.hist.copy())
        if dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        self.hist = t.numpy() + (1 if _env_rank("VH_DRY_BAD_SUM") else 0)

    def cohort_hist(self):
        return self.hist.astype(np.uint64)

    def sync(self):
        pass

    def reset_timers(self):
        self.timers = {k: (0.0, 0) for k in KERNELS}

    def kernel_time(self, name):
        ms, n = self.timers.get(name, (0.0, 0))
        return ms, n, 0.0

    def study_times(self):
        return np.zeros(self.shape[0], np.float64)

    def download(self, n4=False, maps=True):
        return None, None, None, None, [_Result() for _ in range(self.shape[0])]

    def close(self):
        pass


class Pipe:
    """vh_pipe's host side as far as bench.host_to_host sees it: copies through and the
    page-locking budget rule of vh_pipe_run (api.hip: VH_PIPE_PIN_CAP, else 32 GiB per node divided
    by LOCAL_WORLD_SIZE): the caller bytes past the budget count as staged ranges."""

    def __init__(self, R, C, Z, sub, slots=3, device=0):
        self.sub, self.slots = int(sub), int(slots)
        local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
        self.cap = int(os.environ.get("VH_PIPE_PIN_CAP", PIN_NODE_BUDGET // local))
        self.peak, self.staged = 0, 0

    def run(self, hp, mask, opts, n4=True, maps=True, out=None):
        n = hp.shape[0]
        caller = [hp, mask] + [a for a in (out or ()) if a is not None]
        pinned, staged = 0, 0
        for a in caller:
            for i in range(0, n, self.sub):   # one range per sub-batch chunk of each array
                b = a[i:i + self.sub].nbytes
                if pinned + b <= self.cap:
                    pinned += b
                else:
                    staged += 1
        self.peak, self.staged = pinned, staged
        time.sleep(0.002 * ((n + self.sub - 1) // self.sub))   # a nonzero duration per sub-batch
        if out is not None and out[0] is not None:
            out[0][...] = hp
        return (*(out or (None,) * 4), [_Result() for _ in range(n)])

    def stats(self):
        return self.peak, self.staged

    def close(self):
        pass
