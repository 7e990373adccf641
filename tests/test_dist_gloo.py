"""CPU, world size 2 over gloo: bench.py's multi-GPU host logic -- distinct shards per rank, the
RCCL unique-id broadcast, max-over-ranks timing -- and the cohort-histogram semantics the RCCL
all-reduce implements (integer sum of per-rank histograms = histogram of the whole cohort)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import vdp_oracle as O
from vent_analysis_amd.synth import synth_batch

BINS = 1024
SHAPE = (40, 40, 12)
PER_RANK = 3


def cohort_hist(X, M):
    """1024-bin histogram of p99-normalised masked values in [0, 1.5) (vh_run_opts.do_cohort)."""
    h = np.zeros(BINS, np.int64)
    for x, m in zip(X, M):
        s = np.sort(x[m > 0])
        p99 = s[int(len(s) * 0.99)]
        nv = (x / np.float32(p99)).astype(np.float32)[m > 0]
        sel = (nv >= 0) & (nv < np.float32(1.5))
        b = np.minimum((nv[sel] * np.float32(BINS / 1.5)).astype(np.int64), BINS - 1)
        h += np.bincount(b, minlength=BINS)
    return h


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = bench.broadcast_uid(bytes(range(128)) if rank == 0 else None, dist)
    X, M = synth_batch(*SHAPE, PER_RANK, base_seed=bench.shard_seed(rank))
    h = torch.from_numpy(cohort_hist(X, M))
    dist.all_reduce(h, op=dist.ReduceOp.SUM)
    dt = bench.max_over_ranks(0.5 + rank, dist)
    out.put((rank, uid, h.numpy(), dt, [O.mean_f32(x[m > 0]) for x, m in zip(X, M)]))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_shards_uid_timing_and_cohort():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, uid0, h0, dt0, m0), (_, uid1, h1, dt1, m1) = got
    assert uid0 == uid1 == bytes(range(128))
    assert dt0 == dt1 == 1.5                      # slowest rank
    assert np.array_equal(h0, h1)
    assert m0 != m1                               # distinct studies per rank
    Xa, Ma = synth_batch(*SHAPE, PER_RANK, base_seed=bench.shard_seed(0))
    Xb, Mb = synth_batch(*SHAPE, PER_RANK, base_seed=bench.shard_seed(1))
    whole = cohort_hist(np.concatenate([Xa, Xb]), np.concatenate([Ma, Mb]))
    assert np.array_equal(h0, whole)
