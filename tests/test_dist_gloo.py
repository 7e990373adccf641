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


def _bench(cmd, env=None, timeout=300):
    import subprocess
    import sys
    e = dict(os.environ, **(env or {}))
    return subprocess.run([sys.executable] + cmd, cwd=bench.HERE, env=e, capture_output=True,
                          text=True, timeout=timeout)


DRY = ["--dry-run", "--steps", "2", "--warmup", "1", "--batch", str(PER_RANK), "--shape",
       *map(str, SHAPE), "--inflight", "2", "--iso-runs", "2", "--h2h-batches", "2", "--h2h-sub", "2",
       "--h2h-slots", "2"]


def _check_dry_line(out, world, pin_cap=None):
    """bench.main()'s own N > 1 line, produced with tests/standin_lib.py in place of libventhip
    (VERDICT r5 item 1): everything but the device work and RCCL itself ran as on the GPU boxes."""
    import json
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out          # rank 0's one JSON line, nothing else on stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["config"]["parallelism"] == f"dp{world}"
    assert line["data"].startswith("DRY RUN")
    assert line["value"] > 0 and line["steps"] == 2 and line["cpu_baseline"] is None
    X, M = [], []
    for r in range(world):   # each rank's batch 0 (checked after the timed region)
        x, m = synth_batch(*SHAPE, PER_RANK, base_seed=bench.shard_seed(r), vary=True)
        X.append(x)
        M.append(m)
    whole = cohort_hist(np.concatenate(X), np.concatenate(M))
    # the communicator as main() checked it: ranks as the stand-in reported them, the all-reduce
    # checked against the gloo sum of every rank's rows (check_cohort), the cohort's total
    c = line["comm"]
    assert c["kind"].startswith("gloo stand-in")
    assert c["rccl_ranks"] == world and c["rccl_rank"] == 0
    assert c["allreduce_ok"] is True
    assert c["cohort_total"] == int(whole.sum())
    assert len(line["per_rank_vol_s"]) == world and min(line["per_rank_vol_s"]) > 0
    # the roofline block: the dominant class by time per step (10 x 1 ms of n4_pcg beat one 5 ms
    # sort launch), bytes per launch = the class's bytes per step / launches per step
    r = line["roofline"]
    assert r["kernel"] == "n4_pcg" and r["launches_per_step"] == 10.0
    assert r["avg_launch_us"] == 1000.0
    assert r["traffic"] is None and "stale" in r["traffic_note"]
    # the host-to-host leg: slowest rank's median, this rank's page-locking budget
    h = line["host_to_host"]
    assert h["seconds_statistic"] == "max over ranks of each rank's median"
    budget = pin_cap if pin_cap is not None else (32 << 30) // world
    assert h["pin_budget_bytes"] == budget and h["pinned_peak_bytes"] <= budget
    if pin_cap is not None:
        assert h["staged_spans"] > 0
    return line


@pytest.mark.parametrize("world", [2, 3])
def test_bench_gpus_n_launches_n_ranks(world):
    """python bench.py --gpus N (no WORLD_SIZE, the driver's N = 1 command form) starts N ranks
    itself: rank 0's single JSON line carries n_gpus = N, dpN, and the cohort sum of all shards."""
    r = _bench(["bench.py", "--gpus", str(world)] + DRY)
    assert r.returncode == 0, r.stderr[-2000:]
    _check_dry_line(r.stdout, world)


def test_bench_under_torchrun():
    """The torchrun form (WORLD_SIZE from the launcher) gives the same line."""
    r = _bench(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
                "--gpus", "2"] + DRY)
    assert r.returncode == 0, r.stderr[-2000:]
    _check_dry_line(r.stdout, 2)


def test_bench_pin_budget_per_rank():
    """A per-rank page-locking cap past which the pipe stages (VH_PIPE_PIN_CAP) reaches every rank."""
    r = _bench(["bench.py", "--gpus", "2"] + DRY, env={"VH_PIPE_PIN_CAP": str(1 << 16)})
    assert r.returncode == 0, r.stderr[-2000:]
    _check_dry_line(r.stdout, 2, pin_cap=1 << 16)


def test_bench_rank_failure_and_world_mismatch():
    r = _bench(["bench.py", "--gpus", "2"] + DRY, env={"VH_DRY_FAIL_RANK": "1"})
    assert r.returncode != 0
    assert not r.stdout.strip()
    r = _bench(["bench.py", "--gpus", "2"] + DRY, env={"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE 1 but --gpus 2" in r.stderr


@pytest.mark.parametrize("world", [2, 3])
def test_bench_cohort_mismatch_fails(world):
    """A rank whose communicator returns a wrong sum fails the whole job (main()'s check_cohort)."""
    r = _bench(["bench.py", "--gpus", str(world)] + DRY, env={"VH_DRY_BAD_SUM": str(world - 1)})
    assert r.returncode != 0
    assert "differs from the sum" in r.stderr


@pytest.mark.parametrize("world", [2, 3])
def test_bench_communicator_rank_count_checked(world):
    """A communicator that reports the wrong rank count stops the job before the timed region."""
    r = _bench(["bench.py", "--gpus", str(world)] + DRY, env={"VH_DRY_BAD_RANKS": "1"})
    assert r.returncode != 0
    assert "RCCL reports rank 1 of" in r.stderr
