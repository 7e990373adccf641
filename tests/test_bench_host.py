"""CPU: bench.py's roofline bookkeeping -- the dominant kernel class is chosen
by time per step, bytes per launch divide the class's bytes per step by its launches, and a PMC
summary prices a line's traffic only when it was measured on the same library AND workload."""
import json
import os

import numpy as np

import bench


def test_dominant_class_by_time_per_step():
    # config 5's shape of the problem: ~170 grid-PC launches of 0.9 ms against one 1.3 ms sort
    ms = {"n4_pcg": 5 * 170 * 0.9, "sort": 5 * 1.33, "n4_fit": 5 * 170 * 0.46}
    n = {"n4_pcg": 5 * 170, "sort": 5, "n4_fit": 5 * 170}
    dom, per_launch, per_step = bench.dominant_class(ms, n, 5)
    assert dom == "n4_pcg"
    assert abs(per_launch - 0.9) < 1e-12 and per_step == 170


def _summary(path, sha, workload, kernels):
    d = {"lib_sha256": sha, "kernels": kernels}
    if workload is not None:
        d["workload"] = workload
    json.dump(d, open(path, "w"))


def test_pmc_traffic_keyed_by_library_and_workload(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    os.makedirs(tmp_path / "profiles")
    p = bench.make_parser()
    default = bench.workload_key(p.parse_args([]))
    cfg5 = bench.workload_key(p.parse_args(["--shape", "512", "512", "512", "--batch", "1",
                                            "--morph3d"]))
    assert default != cfg5
    k = {"sort": {"traffic_bytes_per_launch": 7.9e8}}
    # an old summary (no workload recorded: the default bench) and a newer one of config 5
    _summary(tmp_path / "profiles" / "r5a_pmc_traffic.json", "abc", None, k)
    _summary(tmp_path / "profiles" / "r6a_pmc_traffic.json", "abc", cfg5,
             {"n4_pcg": {"traffic_bytes_per_launch": 5.0e8}})
    t, src, why = bench.pmc_traffic("sort", default, digest="abc")
    assert t == 7.9e8 and src.endswith("r5a_pmc_traffic.json")
    # config 5's line never takes the default bench's sort traffic (the r5 mistake)
    t, src, why = bench.pmc_traffic("sort", cfg5, digest="abc")
    assert t is None and "not in the summary" in why and src.endswith("r6a_pmc_traffic.json")
    t, _, _ = bench.pmc_traffic("n4_pcg", cfg5, digest="abc")
    assert t == 5.0e8
    # another workload of the same library: refused; another library: stale
    cfg2 = bench.workload_key(p.parse_args(["--shape", "256", "256", "24", "--batch", "1"]))
    t, _, why = bench.pmc_traffic("n4_pcg", cfg2, digest="abc")
    assert t is None and why.startswith("refused")
    t, _, why = bench.pmc_traffic("sort", default, digest="zzz")
    assert t is None and why.startswith("stale")


def test_algorithmic_bytes_per_launch_of_multi_launch_class():
    """n4_pcg's bytes per step are per iteration x masked voxels; per launch divides by the
    launches (one per iteration), so a launch prices 16 B per masked voxel."""
    from types import SimpleNamespace
    R, C, Z = 16, 16, 4
    mk = np.zeros((1, R, C, Z), np.uint8)
    mk[0, 4:12, 4:12, :] = 1
    hp = np.ones_like(mk, dtype=np.float32)
    res = [SimpleNamespace(n4_iters=[10, 5, 3, 2, 0, 0, 0, 0])]
    tot = bench.algorithmic_bytes("n4_pcg", hp, mk, res, R, C, Z, study=False)
    assert tot / 20 == 16.0 * int(mk.sum())
