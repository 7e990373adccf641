"""bench.py -- end-to-end calculate_VDP throughput on MI355X (BASELINE.json metric).

One step = the whole Vent_Analysis.calculate_VDP hot path (N4 with SimpleITK defaults -> sorted
masked list -> numpy-order mean anchor -> threshold + 3x3 median + border -> 99th-pct linear
binning -> k-means -> SNR -> scalars, plus the cohort histogram) over one batch of synthetic
128x128x24 studies already resident in HBM.  N GPUs = N processes (torchrun), each with its own
batch (weak scaling, no data-path collective); the cohort histogram is all-reduced over RCCL once
per step when N > 1.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "volumes/sec end-to-end VDP, 128×128×24 Xe volume, 1 GPU and 8-GPU batch"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# synthetic batch: 64 distinct studies per rank, each with its own lung geometry (masked voxels vary
# by about +-20 %, so the one-workgroup-per-study N4 sees unequal studies; synth.py vary=True)
BENCH_UNIQUE = 64


# ------------------------------------------------------------------------------------------------
# CPU baseline: the oracle (numpy VDP chain + C N4 restatement) on a bounded sample, spawn pool
# ------------------------------------------------------------------------------------------------
def _cpu_one(args):
    R, C, Z, seed = args
    from oracle import native, vdp_oracle as O
    from vent_analysis_amd.synth import synth_volume
    X, M = synth_volume(R, C, Z, seed, True)   # the GPU line's heterogeneous studies (vary=True)
    t = time.perf_counter()
    n4, _, _ = native.n4(X, M)
    O.calculate_vdp(n4, M, (1.5, 1.5, 10.0), HP=X)
    return time.perf_counter() - t


def host_cpu_share():
    """(CPUs this process may use, why).  os.cpu_count() is the whole machine; the affinity mask,
    a cgroup CPU quota and the pool's per-GPU share (OMP_NUM_THREADS, 16 on the GPU boxes, which
    also cap worker pools at that many processes) can each be smaller."""
    n, why = os.cpu_count() or 1, "os.cpu_count()"
    try:
        a = len(os.sched_getaffinity(0))
        if a < n:
            n, why = a, "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(q) // int(per) < n:
            n, why = max(1, int(q) // int(per)), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, why = int(omp), "OMP_NUM_THREADS (the box's CPU share per GPU)"
    return n, why


def cpu_baseline(R, C, Z, seconds=15.0, procs=None, base_seed=0, unique=64):
    """The CPU restatement (C N4 + numpy chain) over the same heterogeneous studies the GPU line
    times (seeds base_seed + i % unique, vary=True), one process per usable host core
    (host_cpu_share), before any GPU initialisation.  Reports per-core throughput and its
    extrapolation to every CPU of the host next to the measured value."""
    import multiprocessing as mp
    from oracle import native
    native.build()
    share, why = host_cpu_share()
    procs = max(1, min(procs or share, share))
    ctx = mp.get_context("spawn")
    done = 0
    busy = 0.0
    with ctx.Pool(procs) as pool:
        pool.map(_cpu_one, [(R, C, Z, base_seed + i % unique) for i in range(procs)])   # warm imports
        t0 = time.perf_counter()
        i = 0
        while time.perf_counter() - t0 < seconds:
            ts = pool.map(_cpu_one, [(R, C, Z, base_seed + (i + j) % unique) for j in range(procs)])
            i += procs
            done += len(ts)
            busy += sum(ts)
        wall = time.perf_counter() - t0
    host = os.cpu_count() or procs
    per_core = done / wall / procs
    return {"value": done / wall, "unit": "volumes/s", "cores": procs, "host_cpus": host,
            "cores_reason": why, "per_core_vol_s": round(per_core, 3),
            "full_host_extrapolated_vol_s": round(per_core * host, 1),
            "kind": "port",
            "sample": f"{done} synthetic {R}x{C}x{Z} volumes, the GPU line's heterogeneous studies "
                      f"(synth_volume vary=True, seeds {base_seed}+i%{unique}; oracle/n4_oracle.c N4, "
                      f"conv_mode 0 = ITK float Welford, + oracle/vdp_oracle.py chain), {procs} "
                      f"processes ({why}) of {host} host CPUs, {wall:.1f} s wall, "
                      f"{busy / max(done, 1):.3f} s per volume per core"}


# ------------------------------------------------------------------------------------------------
# algorithmic bytes per kernel class (DESIGN.md "Roofline accounting")
# ------------------------------------------------------------------------------------------------
def algorithmic_bytes(name, hp, mk, res, R, C, Z, study=True, conv_mode=0):
    """Total algorithmic HBM bytes moved by all launches of kernel class ``name`` in one step.

    N4 state is compact (mask == 1 voxels only, DESIGN.md "HBM layout"), so the per-unit figures
    are per masked voxel and per executed iteration; a volume is only touched by an iteration's
    sweeps while it is still iterating, so the iteration count is the volume's own."""
    V = R * C * Z
    B = hp.shape[0]
    m = mk.reshape(B, R, C * Z)
    vm = (m == 1).sum(axis=(1, 2)).astype(np.float64)          # masked (mask == 1) voxels
    nz = m != 0
    has = nz.any(axis=1)
    lo = np.where(has, nz.argmax(axis=1), 0)
    hi = np.where(has, R - 1 - nz[:, ::-1, :].argmax(axis=1), -1)
    vr = np.maximum(hi - lo + 1, 0).sum(axis=1).astype(np.float64)   # voxels in column ranges
    iters = np.array([sum(r.n4_iters[:4]) for r in res], np.float64)
    levels = np.array([sum(1 for k in range(4) if r.n4_iters[k] > 0) for r in res], np.float64)
    cw = 8.0 if conv_mode == 0 else 0.0   # S7: the field differences d written once, read once
    if name == "n4_eval":        # read ridx + L0 + T windows, write U (+ d, compact order)
        return float(np.sum(iters * (12.0 + cw / 2) * vm))
    if name == "n4_fit":         # read ridx + U
        return float(np.sum(iters * 8.0 * vm))
    if name == "n4_hist":        # read U
        return float(np.sum(iters * 4.0 * vm))
    if name == "n4_study":       # init: read I, write L0 + U; per iteration: hist reads U, fit
        return float(np.sum(iters * (16.0 + cw) * vm + 12.0 * vm))   # reads U, eval L0 in, U out
    if name == "n4_welford":     # read perm + d (raster walk of the compact d)
        return float(np.sum(iters * 8.0 * vm))
    if name in ("n4_pcw", "n4_pcg"):   # pass 0: read perm + d, write p; rounds re-read p (once)
        return float(np.sum(iters * 16.0 * vm))
    if name == "n4_den":         # read ridx, once per level
        return float(np.sum(levels * 4.0 * vm))
    if name == "n4_init":        # row masks / offsets from the column bitmaps (+ the sweep
        tiles = (C * Z + 63) // 64   # driver's init: read I at masked voxels, write L0, U, ridx)
        return float(B * (V / 8.0 + 12.0 * R * tiles) + (0.0 if study else np.sum(16.0 * vm)))
    if name == "n4_final":       # read I, write N4HPvent (every voxel) + the sort keys (masked)
        return float(B * 8.0 * V + np.sum(4.0 * vm))
    if name == "classify":       # write defect, border, LB at every voxel; read N4 + mask only in
        return float(np.sum(3.0 * V + 5.0 * vr))   # the columns' masked row ranges (k_plane skips the rest)
    if name == "mean":           # numpy-order chunk sums + p99: read the sorted masked keys
        return float(np.sum(4.0 * (m != 0).sum(axis=(1, 2))))
    if name == "sort":           # digit histograms (read) + 4 LSD passes (read + write), masked
        return float(np.sum(36.0 * vm))
    if name == "gather":
        return float(np.sum(vr * 5.0 + 4.0 * vm))
    if name == "snr":
        return float(B * 5.0 * V)
    if name == "mask_stats":
        return float(B * 1.0 * V)
    return 0.0


_OWN_LIB = object()


def lib_digest(path=_OWN_LIB):
    """sha256 of the libventhip.so this process runs (vent_analysis_amd/_lib.LIB_PATH), or of
    ``path``; None for a surface with no shared object (the dry run's stand-in: LIB_PATH None)."""
    import hashlib
    if path is _OWN_LIB:
        from vent_analysis_amd import _lib
        path = getattr(_lib, "LIB_PATH", None)
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except (OSError, TypeError):
        return None


DEFAULT_WORKLOAD = None   # filled lazily: workload_key of the default command line


def summary_workload(d):
    """The workload a PMC summary was measured on.  Summaries from before round 6 carry none: they
    were all made by scripts/gpu_pmc.sh on the default bench command line."""
    global DEFAULT_WORKLOAD
    if DEFAULT_WORKLOAD is None:
        DEFAULT_WORKLOAD = workload_key(make_parser().parse_args([]))
    return d.get("workload") or DEFAULT_WORKLOAD


def pmc_traffic(kernel, workload, digest=_OWN_LIB):
    """Per-launch HBM-side bytes of ``kernel`` from the newest committed PMC summary
    (profiles/r*_pmc_traffic.json, written by scripts/pmc_summary.py from separate rocprofv3 --pmc
    passes) of this very library (its sha256) AND this very workload (workload_key: shape, batch,
    driver and N4 options).  The bench cannot collect PMC counters itself (rocprofv3 wraps the
    process).  Returns (bytes or None, source file or None, why)."""
    import glob
    def run_order(f):   # r<round><tag>: tags run a..z, then aa..az, ... (r4z before r4av)
        m = re.match(r"r(\d+)([a-z]*)", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_pmc_traffic.json")), key=run_order)
    if not files:
        return None, None, "no committed PMC summary"
    mine = lib_digest() if digest is _OWN_LIB else digest
    if mine is None:   # no shared object to match (the dry run's stand-in)
        return None, None, "stale: no library digest, no summary can match"
    same_lib = None
    for f in reversed(files):   # the newest summary of this library and workload
        d = json.load(open(f))
        if d.get("lib_sha256") != mine:
            continue
        same_lib = same_lib or f
        if summary_workload(d) != workload:
            continue
        src = os.path.relpath(f, HERE)
        k = d["kernels"].get(kernel)
        if not k:
            return None, src, f"{kernel} not in the summary of this library and workload"
        return k["traffic_bytes_per_launch"], src, "same library (sha256) and workload"
    if same_lib:
        return None, os.path.relpath(same_lib, HERE), ("refused: the summaries of this library were "
                                                       "measured on another workload")
    src = os.path.relpath(files[-1], HERE)
    d = json.load(open(files[-1]))
    return None, src, (f"stale: no summary of this run's library {str(mine)[:12]} (newest: "
                       f"{str(d.get('lib_sha256'))[:12]})")


def dominant_class(iso_ms_total, iso_launches, runs):
    """The kernel class with the most time per step when batch 0 runs alone: each class's summed
    launch time over ``runs`` isolated runs, divided by the runs (launch time x launches per step).
    Returns (class, mean launch ms, launches per step)."""
    per_step = {k: iso_ms_total[k] / runs for k in iso_ms_total if iso_launches.get(k)}
    dom = max(per_step, key=lambda k: per_step[k])
    return dom, iso_ms_total[dom] / iso_launches[dom], iso_launches[dom] / runs


# ------------------------------------------------------------------------------------------------
# distributed host logic (one process per GPU; tests/test_dist_gloo.py runs it on gloo)
# ------------------------------------------------------------------------------------------------
def shard_seed(rank):
    """Base seed of a rank's synthetic batch: each rank owns distinct studies (weak scaling)."""
    return 1000 * rank


def broadcast_uid(uid, dist):
    """Rank 0's RCCL unique id to every rank (uid is ignored on ranks > 0)."""
    box = [uid if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def max_over_ranks(dt, dist):
    """The job's step time is the slowest rank's."""
    import torch
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def check_cohort(local, reduced, dist):
    """N > 1 self-check of the cohort all-reduce: the histogram the communicator summed must equal
    the per-rank histograms summed over gloo (an independent path).  Every rank learns the verdict
    (MIN over ranks), so a mismatch on any rank fails every rank."""
    import torch
    g = torch.from_numpy(np.ascontiguousarray(local, dtype=np.int64))
    dist.all_reduce(g, op=dist.ReduceOp.SUM)
    mine = int(np.array_equal(np.asarray(reduced, dtype=np.int64), g.numpy()))
    ok = torch.tensor([mine], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return bool(ok.item()), int(g.numpy().sum())


def per_rank(value, dist):
    """Every rank's value of a per-rank quantity, in rank order (gloo all_gather)."""
    import torch
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(dist.get_world_size())]
    dist.all_gather(out, torch.tensor([float(value)], dtype=torch.float64))
    return [float(t.item()) for t in out]


class stdout_to_stderr:
    """RCCL's communicator setup prints a version banner on stdout; rank 0's stdout must carry the
    one JSON line only (the driver parses it), so fd 1 points at fd 2 while the block runs."""
    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def host_to_host(R, C, Z, nb, args, device, opts, seed, aligned=True, _lib=None):
    """Volumes/s from host memory to host memory: args.h2h_batches x nb studies streamed through
    vh_pipe in sub-batches of args.h2h_sub studies on args.h2h_slots slots (pinned staging, one
    stream each: the H2D, compute and D2H of different sub-batches overlap, and the studies of
    concurrent sub-batches fill the CUs that finished studies free), inputs HPvent + mask in,
    every output the class returns out (N4HPvent, defectArray, defectBorder, defectArrayLB,
    scalars).  The slowest rank's time is what the caller's aggregate uses (ranks run
    independently)."""
    if _lib is None:
        from vent_analysis_amd import _lib
    from vent_analysis_amd.synth import synth_batch
    slots, sub = args.h2h_slots, min(args.h2h_sub, nb)
    hb = args.h2h_batches or (12 if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 6)
    n = max(1, hb) * nb
    hp0, mk0 = synth_batch(R, C, Z, n, base_seed=seed, unique=BENCH_UNIQUE, vary=True)
    # page-aligned host arrays (as ingest.load_batch allocates them): whole chunks DMA in place
    alloc = _lib.empty_aligned if aligned else (lambda shape, t: np.empty(shape, t))
    hp, mk = alloc(hp0.shape, np.float32), alloc(mk0.shape, np.uint8)
    hp[...] = hp0
    mk[...] = mk0
    del hp0, mk0
    P = _lib.Pipe(R, C, Z, sub, slots=slots, device=device)
    out = tuple(alloc(hp.shape, t) for t in (np.float32, np.uint8, np.uint8, np.uint8))
    P.run(hp[:slots * sub], mk[:slots * sub], opts,
          out=tuple(a[:slots * sub] for a in out))          # warm: every slot's workspaces
    runs = []
    for _ in range(3):   # the median of three passes (the first one also first-touches the outputs)
        t = time.perf_counter()
        P.run(hp, mk, opts, out=out)
        runs.append(time.perf_counter() - t)
    pinned_peak, staged = P.stats()
    P.close()
    budget = pin_budget()
    if pinned_peak > budget:
        raise RuntimeError(f"vh_pipe pinned {pinned_peak} B in place, past this rank's budget {budget} B")
    dt = sorted(runs)[1]
    return {"volumes": n, "seconds": round(dt, 6), "runs_seconds": [round(r, 6) for r in runs],
            "statistic": "median of 3 passes", "sub_batch": sub, "slots": slots,
            "pinned_peak_bytes": pinned_peak, "pin_budget_bytes": budget, "staged_spans": staged,
            "includes": "H2D of HPvent f32 + mask u8, the full pipeline, D2H of N4HPvent f32 + "
                        "defect / border / LB u8 + per-study scalars, host staging memcpys; over "
                        "PCIe the mask travels as bits and the three maps as one packed byte "
                        "(packed / unpacked on host threads inside the timed region)",
            "bytes_per_volume": int(R * C * Z * (4 + 1 + 4 + 3)),
            "pcie_bytes_per_volume": int(R * C * Z * (4 + 0.125 + 4 + 1))}


def pin_budget():
    """This rank's vh_pipe_run page-locking budget, by the library's rule (api.hip, vh_pipe_create):
    VH_PIPE_PIN_CAP bytes, else 32 GiB per node divided by LOCAL_WORLD_SIZE (the ranks sharing
    the host's memory)."""
    if os.environ.get("VH_PIPE_PIN_CAP"):
        return int(os.environ["VH_PIPE_PIN_CAP"])
    return (32 << 30) // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))


def link_probe(device, mb=256, _lib=None):
    """This box's PCIe link with pinned host memory: H2D alone, D2H alone and both at once on two
    streams (as the pipe's overlapped chunks use it), best of 3 each (vh_link_probe).  The
    host-to-host line can not beat link rate / PCIe bytes per volume, whatever the device rate."""
    if _lib is None:
        from vent_analysis_amd import _lib
    r = _lib.context(device).link_probe(mb << 20)
    r["bytes_each_way"] = mb << 20
    return r


def link_bound(link, R, C, Z):
    """Upper bound of the host-to-host rate from the link probe: the pipe moves 4.125 bytes per
    voxel in (HPvent f32, mask bits) and 5 out (N4HPvent f32, one packed map byte)."""
    v = R * C * Z
    b_in, b_out = v * 4.125, v * 5.0
    return min(link["both_GBps"] * 1e9 / (b_in + b_out), link["h2d_GBps"] * 1e9 / b_in,
               link["d2h_GBps"] * 1e9 / b_out)


def main_ci(args):
    """CI line: defect-voxels/s and sphere-probes/s of the cluster-index map
    on 128x128x24 studies, host-to-host through vh_ci (defect map in, float64 CI map out).  Two
    inputs: the seed-0 study's defect map from the GPU pipeline itself (5917 defect voxels, CI
    22.5: the study BASELINE.md timed at 44.4 s), and a random clustered map of ~6 000 defects."""
    from vent_analysis_amd import _lib
    from vent_analysis_amd.sphere import compact_table, sphere_pix
    from vent_analysis_amd.synth import synth_volume
    R, C, Z = 128, 128, 24
    vox = (1.5, 1.5, 10.0)
    X, M = synth_volume(R, C, Z, 0)
    Bt = _lib.Batch(R, C, Z, 1)
    Bt.upload(X[None], M.astype(np.uint8)[None])
    Bt.run(Bt.options(do_n4=True, vox=vox))
    _, d0, _, _, _ = Bt.download(n4=False)
    Bt.close()
    rng = np.random.default_rng(0)
    i, j, k = np.meshgrid(np.arange(R), np.arange(C), np.arange(Z), indexing="ij")
    blobs = np.zeros((R, C, Z), bool)
    while blobs.sum() < 5900:
        c = [rng.uniform(0.15, 0.85) * s for s in (R, C, Z)]
        r = rng.uniform(4, 9)
        blobs |= ((i - c[0]) ** 2 + (j - c[1]) ** 2 + ((k - c[2]) * 6.67) ** 2 <= r * r) & (M > 0)
    table = compact_table(sphere_pix(vox, 50), (R, C, Z))
    cases = {}
    for name, d in (("seed0_pipeline", d0[0]), ("clustered", blobs)):
        d = d.astype(np.uint8)
        # the shells (for the probe count) once, untimed; the timed calls return what
        # CI.calculate_CI returns: the float64 map and the 95th-percentile CI
        _, _, shell = _lib.ci(d, table, float(np.min(vox)))
        for _ in range(max(1, args.warmup)):
            ci, sc, _ = _lib.ci(d, table, float(np.min(vox)), shell=False)
        if not args.no_profile:
            _lib.ctx_profile(True)
        t = time.perf_counter()
        for _ in range(args.steps):
            ci, sc, _ = _lib.ci(d, table, float(np.min(vox)), shell=False)
        dt = (time.perf_counter() - t) / args.steps
        kms, kn = _lib.ctx_kernel_time("ci_walk") if not args.no_profile else (0.0, 0)
        _lib.ctx_profile(False)
        nd = int((d > 0).sum())
        probes = int(np.sum(table.bounds[shell[0][d > 0]].astype(np.int64)))
        cases[name] = {"defect_voxels": nd, "seconds_per_map": round(dt, 6),
                       "defect_voxels_per_s": round(nd / dt, 1), "sphere_probes_per_s": round(probes / dt, 1),
                       "sphere_probes": probes, "CI": float(sc[0]),
                       "ci_walk_us": round(kms / kn * 1e3, 2) if kn else None}
    head = cases["seed0_pipeline"]   # 5917 defects, CI 22.5: the study BASELINE.md timed
    roof = None
    if head["ci_walk_us"]:
        # k_ci_walk is bound by LDS bit tests, not HBM: each sphere probe is one
        # ds_read_b32 of the LDS-staged defect bitmap (4 B); peak = 128 B/clk/CU (ds_read_b32,
        # MI355X_MICROARCH.md LDS table) x 256 CUs x 2.4 GHz
        lds_peak = 128.0 * 256 * 2.4e9 / 1e9
        ach = head["sphere_probes"] * 4.0 / (head["ci_walk_us"] * 1e-6) / 1e9
        roof = {"bound": "lds", "kernel": "ci_walk", "achieved": round(ach, 1), "peak": lds_peak,
                "unit": "GB/s", "frac": round(ach / lds_peak, 4), "traffic": None,
                "avg_launch_us": head["ci_walk_us"],
                "probes_per_s_kernel": round(head["sphere_probes"] / (head["ci_walk_us"] * 1e-6), 1),
                "alg_bytes_per_launch": head["sphere_probes"] * 4.0}
    line = {"metric": "CI defect-voxels/s (cluster-index map, 128x128x24, host-to-host)",
            "value": head["defect_voxels_per_s"], "unit": "defect-voxels/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(head["seconds_per_map"] * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(head["defect_voxels_per_s"] / (5917 / 44.4), 1),
            "dtype": "u8/f64", "data": "synthetic",
            "config": {"workload": "CI.calculate_CI + the 95th-percentile CI on one 128x128x24 "
                                   "study, Rmax 50, vox [1.5, 1.5, 10]", "cases": cases},
            "roofline": roof, "cpu_baseline": None,
            "baseline_note": "reference: 5917 clustered defect voxels in 44.4 s (BASELINE.md)"}
    print(json.dumps(line))


def main_class(args):
    """One-study latency line: Vent_Analysis.calculate_VDP -- the GUI's call --
    on one synthetic study of --shape, host arrays in and out (H2D, N4 on the grid form, the VDP
    chain, D2H of N4HPvent and the three maps, the class's numpy bookkeeping), args.steps calls
    after args.warmup, the median call reported.  The study's own device batch is pooled
    (_lib.pooled_batch), as in an interactive session that analyses study after study."""
    import contextlib
    import io
    from vent_analysis_amd import Vent_Analysis
    from vent_analysis_amd.synth import synth_volume
    R, C, Z = args.shape
    X, M = synth_volume(R, C, Z, 0, True)
    vox = (1.5, 1.5, 10.0)
    ts = []
    sink = io.StringIO()   # the class prints the reference's status lines; stdout carries the JSON
    for i in range(args.warmup + args.steps):
        with contextlib.redirect_stdout(sink):
            v = Vent_Analysis(xenon_array=X, mask_array=M, vox=vox)
            t = time.perf_counter()
            v.calculate_VDP()
        if i >= args.warmup:
            ts.append(time.perf_counter() - t)
    med = sorted(ts)[len(ts) // 2]
    line = {"metric": f"calculate_VDP latency, one {R}x{C}x{Z} study (host to host)",
            "value": round(1.0 / med, 2), "unit": "volumes/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(med * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "Vent_Analysis(xenon_array, mask_array).calculate_VDP(): N4 + "
                                   "mean-anchored + linear-binning + k-means VDP + border + SNR, one "
                                   "study, host arrays in and out", "shape": [R, C, Z],
                       "n4_iterations": [int(i) for i in v.n4_iterations]},
            "latency_ms": {"median": round(med * 1e3, 3), "min": round(min(ts) * 1e3, 3),
                           "max": round(max(ts) * 1e3, 3)},
            "roofline": None, "cpu_baseline": None}
    print(json.dumps(line))


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args, argv):
    """``--gpus N`` (N > 1) without a launcher's WORLD_SIZE: start N rank processes of this script
    (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as torchrun sets
    them) before this process touches any GPU, pass rank 0's stdout (the one JSON line) through,
    and exit non-zero if any rank fails (the others are then stopped).  This process never
    initialises the GPU, so nothing is exec'd from a GPU process."""
    import subprocess
    n = args.gpus
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {procs.index(p)} exited with {c}; stopping the other ranks",
                      file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=256, help="volumes per GPU")
    ap.add_argument("--shape", type=int, nargs=3, default=(128, 128, 24))
    ap.add_argument("--no-n4", action="store_true", help="VDP chain only (N4 := identity)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true",
                    help="no HIP events in the isolated runs (no roofline); the timed region never has any")
    ap.add_argument("--subbatch", type=int, default=0, help="volumes per N4 sub-batch (0: all)")
    ap.add_argument("--n4-mode", default="auto", choices=["auto", "sweep", "study", "grid"],
                    help="N4 driver: per-iteration sweeps, one workgroup per study, or one study "
                         "over a cooperative grid of workgroups")
    ap.add_argument("--morph3d", action="store_true",
                    help="build-defined 3-D median / border (BASELINE config 5)")
    ap.add_argument("--conv-mode", type=int, default=0, choices=[0, 1],
                    help="N4 convergence measure: 0 ITK's float Welford recurrence (SimpleITK "
                         "semantics, default), 1 exact CoV (faster, different iteration counts)")
    ap.add_argument("--comm", action="store_true",
                    help="at --gpus 1: go through the RCCL path anyway (comm_init(1, 0) + one "
                         "cohort all-reduce per step)")
    ap.add_argument("--no-h2h", action="store_true",
                    help="skip the host-to-host pipeline measurement (host_to_host_vol_s)")
    ap.add_argument("--h2h-batches", type=int, default=0,
                    help="host-to-host sample: this many x --batch volumes (0: 12 at one rank, 6 "
                         "per rank beyond: ~14 GB of host arrays per rank at 12)")
    ap.add_argument("--h2h-sub", type=int, default=224,
                    help="host-to-host: studies per pipeline sub-batch")
    ap.add_argument("--h2h-slots", type=int, default=3,
                    help="host-to-host: pipeline slots (sub-batches in flight, <= 8)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="device batches in flight: steps of consecutive batches overlap on their own "
                         "streams (a cohort stream); 1 = one batch, synchronised every step")
    ap.add_argument("--h2h-keep-batch", action="store_true",
                    help="A/B: keep the device-resident batch (and its stream) open during the "
                         "host-to-host measurement (round-3 behaviour)")
    ap.add_argument("--iso-runs", type=int, default=5,
                    help="runs of batch 0 alone after the timed region (batch latency and the "
                         "isolated kernel durations the roofline uses)")
    ap.add_argument("--workload", default="vdp", choices=["vdp", "ci", "class"],
                    help="vdp: the BASELINE metric (default); ci: the cluster-index line; class: "
                         "one study's Vent_Analysis.calculate_VDP latency, host to host")
    ap.add_argument("--dry-run", action="store_true",
                    help="tests only: this main() on the CPU over gloo with tests/standin_lib.py in "
                         "place of libventhip (every host step of the N > 1 line runs; the stand-in's "
                         "cohort all-reduce is a gloo all-reduce); the line says so and measures nothing")
    ap.add_argument("--conv-threshold", type=float, default=0.001,
                    help="N4 convergence threshold (SimpleITK default 0.001; 0 = fixed 4x50 "
                         "iterations, for kernel A/B runs at constant work)")
    return ap


def workload_key(args):
    """What a PMC summary must have been measured on to price this line's traffic: the shape, the
    batch and every option that changes which kernels run or how much work they do."""
    return {"shape": [int(v) for v in args.shape], "batch": int(args.batch),
            "n4_mode": args.n4_mode, "morph3d": bool(args.morph3d), "conv_mode": int(args.conv_mode),
            "conv_threshold": float(args.conv_threshold), "no_n4": bool(args.no_n4),
            "subbatch": int(args.subbatch)}


def load_lib(dry_run):
    """libventhip's ctypes shim, or under --dry-run (tests only) the CPU stand-in with the same
    surface (tests/standin_lib.py)."""
    if dry_run:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import standin_lib
        return standin_lib
    from vent_analysis_amd import _lib
    return _lib


def main():
    args = make_parser().parse_args()
    if args.workload == "ci":
        return main_ci(args)
    if args.workload == "class":
        return main_class(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:   # python bench.py --gpus N: N ranks
        sys.exit(launch_ranks(args, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE {world} but --gpus {args.gpus} (one rank per GPU)")
    R, C, Z = args.shape
    nb = args.batch

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.dry_run:
        cpu = cpu_baseline(R, C, Z, seconds=args.cpu_seconds, base_seed=shard_seed(0),
                           unique=BENCH_UNIQUE)   # before any GPU initialisation

    dist = None
    if world > 1 or args.dry_run:
        import torch.distributed as dist
        with stdout_to_stderr():   # gloo prints its connection banner on fd 1
            dist.init_process_group("gloo", rank=rank, world_size=world)
    _lib = load_lib(args.dry_run)
    from vent_analysis_amd.synth import synth_batch

    # --inflight I: I device batches (distinct studies) whose steps are enqueued back to back on
    # their own streams, so batch i + 1's N4 workgroups take the CUs that batch i's short studies
    # free (a cohort stream); I = 1 is one batch, synchronised every step
    ninf = max(1, args.inflight)
    data, batches = [], []
    for i in range(ninf):
        h_, m_ = synth_batch(R, C, Z, nb, base_seed=shard_seed(rank) + BENCH_UNIQUE * i,
                             unique=BENCH_UNIQUE, vary=True)
        b_ = _lib.Batch(R, C, Z, nb, device=local)
        b_.upload(h_, m_)
        data.append((h_, m_))
        batches.append(b_)
    hp, mk = data[0]
    Bt = batches[0]
    use_comm = world > 1 or args.comm
    comm = None
    with stdout_to_stderr():
        if world > 1:
            uid = broadcast_uid(_lib.comm_unique_id() if rank == 0 else None, dist)
            _lib.comm_init(world, rank, uid, device=local)
        elif args.comm:
            _lib.comm_init(1, 0, _lib.comm_unique_id(), device=local)
        if use_comm:   # what RCCL itself reports (ncclCommCount / ncclCommUserRank)
            n_rccl, r_rccl = _lib.comm_info(device=local)
            comm = {"kind": getattr(_lib, "COMM_KIND", "rccl"), "rccl_ranks": n_rccl,
                    "rccl_rank": r_rccl}
            if n_rccl != world or r_rccl != rank:
                sys.exit(f"bench.py: RCCL reports rank {r_rccl} of {n_rccl}, expected {rank} of {world}")
    vox = (1.5, 1.5, 10.0)
    opts = Bt.options(do_n4=not args.no_n4, vox=vox, do_cohort=True,
                      profile=not args.no_profile, n4_subbatch=args.subbatch,
                      conv_threshold=args.conv_threshold, morph3d=args.morph3d,
                      n4_mode=args.n4_mode, conv_mode=args.conv_mode)
    warm = Bt.options(do_n4=not args.no_n4, vox=vox, do_cohort=True, profile=False,
                      n4_subbatch=args.subbatch, conv_threshold=args.conv_threshold,
                      morph3d=args.morph3d, n4_mode=args.n4_mode, conv_mode=args.conv_mode)

    def step(o, i=0):
        b_ = batches[i % ninf]
        b_.run(o)
        if use_comm:
            b_.cohort_allreduce()
        if ninf == 1:
            b_.sync()

    def sync_all():
        for b_ in batches:
            b_.sync()

    try:
        import torch
        if not args.dry_run and torch.cuda.is_available():   # this rank's GPU (torch's current device is 0 otherwise)
            torch.cuda.set_device(local)
            sync_dev = torch.cuda.synchronize
        else:
            sync_dev = lambda: None  # noqa: E731
    except Exception:   # torch is plumbing only; the library syncs its own stream
        sync_dev = lambda: None  # noqa: E731

    for i in range(args.warmup):
        step(warm, i)
    sync_all()
    for b_ in batches:
        b_.reset_timers()
    if dist:
        dist.barrier()
    sync_dev()
    t0 = time.perf_counter()
    for i in range(args.steps):   # no HIP events in the timed region (they cost a one-study step
        step(warm, i)             # of ~500 short launches half its time): the isolated runs below time kernels
    sync_all()
    sync_dev()
    t_local = time.perf_counter() - t0
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    rates = None
    if dist:
        dt = max_over_ranks(dt, dist)
        rates = per_rank(nb * args.steps / t_local, dist)
    if use_comm:
        # after the timed region: one step of batch 0 without the collective, its local histogram,
        # then RCCL's sum of it checked against the per-rank histograms summed over gloo
        Bt.run(warm)
        Bt.sync()
        loc = Bt.cohort_hist()
        Bt.cohort_allreduce()
        Bt.sync()
        red = Bt.cohort_hist()
        if dist:
            comm["allreduce_ok"], comm["cohort_total"] = check_cohort(loc, red, dist)
        else:   # one rank: the sum over one rank is the local histogram
            comm["allreduce_ok"], comm["cohort_total"] = bool(np.array_equal(loc, red)), int(loc.sum())
    _, _, _, _, res = Bt.download(n4=False, maps=False)
    st_us = Bt.study_times()   # per-study wall time of the last step's one-workgroup-per-study N4
    if os.environ.get("VH_STUDY_TRACE"):   # the other batches' placements too (A/B runs)
        for b_ in batches[1:args.steps]:
            b_.study_times()
    tail = None
    if st_us.max() > 0:
        tail = {"min_us": round(float(st_us.min()), 1), "mean_us": round(float(st_us.mean()), 1),
                "max_us": round(float(st_us.max()), 1),
                "max_over_mean": round(float(st_us.max() / st_us.mean()), 4)}
    batch_latency_ms = None
    iso_kernels = {}   # class -> (summed ms, launches) over the isolated runs of batch 0
    if ninf > 1 or not args.no_profile:
        # batch 0 alone, args.iso_runs times (untimed above): the latency one batch sees, and every
        # kernel class's launch duration with no other batch's workgroups on the CUs -- what a
        # kernel-trace of one batch at a time reports (rocprofv3 --kernel-trace --stats of
        # bench.py --inflight 1), so the roofline fraction is reproducible from profiles/
        Bt.reset_timers()
        lat = []
        for _ in range(max(1, args.iso_runs)):
            t1 = time.perf_counter()
            step(opts, 0)
            sync_all()
            lat.append(time.perf_counter() - t1)
        batch_latency_ms = round(sorted(lat)[len(lat) // 2] * 1e3, 3)
        if not args.no_profile:
            for name in _lib.lib().vh_batch_kernel_names().decode().split(";"):
                ms, n, _ = Bt.kernel_time(name)
                if n:
                    iso_kernels[name] = (ms, n)
    roof = None
    # the volume-resident kernels (one workgroup per study, or the grid form for one study) ran when
    # their timer class did: n4_init then counts only the row scans (algorithmic_bytes)
    used_study = "n4_study" in iso_kernels
    if iso_kernels:
        runs = max(1, args.iso_runs)
        # the dominant class is the one with the most time per step (launch time x launches), not
        # the longest single launch: config 5's ~170 grid-PC launches outweigh its one sort launch
        # vdp_chain is the span of the whole post-N4 chain (several kernels, two streams), not a class
        kern = {n: v for n, v in iso_kernels.items() if n != "vdp_chain"}
        dom, iso_ms, per_step = dominant_class({n: v[0] for n, v in kern.items()},
                                               {n: v[1] for n, v in kern.items()}, runs)
        iso_us = iso_ms * 1e3
        # algorithmic_bytes is the class's total over one step: per launch = / launches per step
        bpl = algorithmic_bytes(dom, hp, mk, res, R, C, Z, study=used_study,
                                conv_mode=args.conv_mode) / per_step
        ach = bpl / (iso_us * 1e-6) / 1e9
        traffic, tsrc, tnote = pmc_traffic(dom, workload_key(args), digest=lib_digest(
            getattr(_lib, "LIB_PATH", None)))
        lim = {"n4_study": "latency, below the HBM roof: the serial S7 recurrence evaluated by "
                           "guess-and-verify rounds and the latency-bound fit / eval walks of one "
                           "workgroup per study (DESIGN.md section 5)",
               "n4_pcg": "latency, below the HBM roof: the serial S7 recurrence of one large study "
                         "by guess-and-verify rounds over a cooperative grid, one grid barrier per "
                         "round (DESIGN.md section 4.2)"}
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": round(traffic) if traffic else None,
                "traffic_source": f"from committed profile {tsrc}" if tsrc else None,
                "traffic_note": tnote,
                "traffic_over_alg": round(traffic / bpl, 3) if traffic else None,
                "avg_launch_us": round(iso_us, 2), "alg_bytes_per_launch": bpl,
                "launches_per_step": round(per_step, 3),
                "dominant_by": "time per step of batch 0 alone (mean launch x launches per step)",
                "timing": f"HIP events around each launch of batch 0 alone, mean of "
                          f"{runs} runs (no other batch on the CUs)",
                "limiter": lim.get(dom),
                "kernel_us_per_launch": {n: round(v[0] / v[1] * 1e3, 2) for n, v in
                                         sorted(kern.items(), key=lambda kv: -kv[1][0])},
                "kernel_us_per_step": {n: round(v[0] / runs * 1e3, 2) for n, v in
                                       sorted(kern.items(), key=lambda kv: -kv[1][0])},
                "non_n4_us_per_step": round(sum(v[0] for n, v in kern.items()
                                                if not n.startswith("n4_")) / runs * 1e3, 2)}
        # non_n4_us_per_step sums the non-N4 kernel classes' launch times; the wall-clock figure is
        # the mask statistics plus the post-N4 chain's span (vdp_chain: its launch gaps included, and
        # k-means beside the mean / cohort on the side stream counted once)
        chain = iso_kernels.get("vdp_chain")
        if chain:
            roof["non_n4_wall_us_per_step"] = round(
                (kern.get("mask_stats", (0.0, 0))[0] + chain[0]) / runs * 1e3, 2)
    its = np.array([list(r.n4_iters[:4]) for r in res])
    if not args.h2h_keep_batch:
        # the device-resident batches (their streams, 1.5 GB of HBM each) are done: the pipe's slot
        # streams then have the GPU_MAX_HW_QUEUES (4) hardware queues to themselves
        for b_ in batches:
            b_.close()
    h2h = None
    if not args.no_h2h:
        if dist:   # every rank streams at once (host memory and PCIe shared as in a cohort run)
            dist.barrier()
        h2h = host_to_host(R, C, Z, nb, args, local, warm, shard_seed(rank) + 500, _lib=_lib)
        h2h["link"] = link_probe(local, _lib=_lib)
        h2h["link"]["bound_vol_s"] = round(link_bound(h2h["link"], R, C, Z), 1)
        h2h["link"]["h2h_of_bound"] = round(h2h["volumes"] / h2h["seconds"] / h2h["link"]["bound_vol_s"], 3)
        if dist:   # the aggregate uses the slowest rank's time
            h2h["seconds"] = round(max_over_ranks(h2h["seconds"], dist), 6)
            h2h["seconds_statistic"] = "max over ranks of each rank's median"
    total = world * nb * args.steps
    line = {
        "metric": METRIC,
        "value": round(total / dt, 2),
        "unit": "volumes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic" if not args.dry_run else
                "DRY RUN: tests/standin_lib.py in place of libventhip (CPU, gloo); nothing measured",
        "config": {"workload": f"batch of {nb} synthetic {R}x{C}x{Z} Xe volumes per GPU, "
                               "end-to-end calculate_VDP: N4 (SimpleITK defaults 4x50 it) + "
                               "mean-anchored + linear-binning + k-means VDP + defect border + "
                               "SNR + cohort histogram" + (" (N4 skipped)" if args.no_n4 else ""),
                   "volumes_per_gpu": nb, "shape": [R, C, Z],
                   "distinct_studies_per_gpu": min(nb, BENCH_UNIQUE) * ninf, "lung_geometry": "per study",
                   "parallelism": f"dp{world}", "n4_subbatch": args.subbatch or nb,
                   "batches_in_flight": ninf,
                   "n4_iterations_mean": float(its.sum(axis=1).mean()) if its.size else 0.0},
        "roofline": roof,
        "cpu_baseline": cpu,
        "n4_study_times": tail,
        "batch_latency_ms": batch_latency_ms if ninf > 1 else round(dt / args.steps * 1e3, 3),
        "host_to_host_vol_s": round(world * h2h["volumes"] / h2h["seconds"], 2) if h2h else None,
        "host_to_host": h2h,
    }
    if comm:
        line["comm"] = comm
    if rates:
        line["per_rank_vol_s"] = [round(r, 2) for r in rates]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm and not comm["allreduce_ok"]:
        sys.exit("bench.py: the RCCL cohort all-reduce differs from the sum of the per-rank histograms")
    if args.h2h_keep_batch:
        for b_ in batches:
            b_.close()
    if use_comm:
        with stdout_to_stderr():
            _lib.comm_destroy(device=local)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    if os.environ.get("VH_DUMP_MAPS"):   # symbolising exit-time faults (scripts/dev): the mappings
        import atexit                     # as they stand when Python's exit handlers run
        atexit.register(lambda: open(os.environ["VH_DUMP_MAPS"], "w").write(open("/proc/self/maps").read()))
    main()
