"""GPU parity tests (MI355X): the HIP path through the C-ABI against the reference goldens and the
CPU oracle.  Tolerances: masks / indices / counts bit-exact; VDP scalars exact (they are ratios of
exact counts); SNR rel 1e-5; N4 rel 1e-5 (north_star), identical iteration counts."""
import hashlib
import os

import numpy as np
import pytest

from conftest import load_case, golden_files
from oracle import native, vdp_oracle as O
from vent_analysis_amd import _lib
from vent_analysis_amd.sphere import compact_table, sphere_pix
from vent_analysis_amd.synth import synth_volume, synth_batch

pytestmark = pytest.mark.gpu

GOLD = golden_files()


def parula():
    """tests/golden/parula.npy: the reference's colour table (/root/reference/parula.npy, a data
    file it ships; screenShot loads it at Vent_Analysis.py:466), loaded without pickle."""
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "parula.npy"), allow_pickle=False)


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)))


def test_library_runs_on_gpu():
    assert _lib.device_count() >= 1
    c = _lib.context(0)
    assert c.h


@pytest.mark.parametrize("path", GOLD, ids=lambda p: p.split("/")[-1])
def test_vdp_chain_vs_reference(path):
    X, M, vox, exp, _ = load_case(path)
    d, bo, lb, res = _lib.vdp(X, M.astype(np.uint8), vox, hp=X)   # N4 = identity, as the goldens
    r = res[0]
    assert np.array_equal(d[0], exp["defect"])
    assert np.array_equal(bo[0] == 1, exp["defect_border"])
    assert np.array_equal(lb[0], exp["lb"])
    assert np.float32(r.mean_anchor) == exp["mean_anchor"]
    assert np.float32(r.p99) == exp["p99"]
    assert 100 * np.float64(r.n_defect) / np.sum(M) == exp["VDP"]
    assert 100 * np.float64(r.n_lb12) / np.sum(M) == exp["VDP_lb"]
    assert r.n_defect * np.prod(np.divide(vox, 10)) / 1000 == exp["DefectVolume"]
    assert r.defect_volume == pytest.approx(exp["DefectVolume"], rel=1e-15)
    assert r.lung_volume == pytest.approx(exp["LungVolume"], rel=1e-15)
    assert rel(np.float32(r.snr), exp["SNR"]) < 1e-5


@pytest.mark.parametrize("path", GOLD, ids=lambda p: p.split("/")[-1])
def test_mask_border_vs_reference(path):
    X, M, vox, exp, _ = load_case(path)
    assert np.array_equal(_lib.border(M.astype(np.uint8))[0], exp["mask_border"])


def test_snr_vs_reference():
    for path in GOLD:
        X, M, vox, exp, _ = load_case(path)
        s = _lib.snr(X, M.astype(np.uint8))[0]
        assert rel(np.float32(s), exp["SNR"]) < 1e-5, path


@pytest.mark.parametrize("path", [p for p in GOLD if "ci_values" in np.load(p)],
                         ids=lambda p: p.split("/")[-1])
def test_ci_vs_reference(path):
    X, M, vox, exp, _ = load_case(path)
    d = exp["defect"]
    table = compact_table(sphere_pix(vox, 50), d.shape)
    ci, sc, shell = _lib.ci(d, table, float(np.min(vox)))
    assert np.array_equal(ci[0][d > 0], exp["ci_values"])
    assert np.all(ci[0][d == 0] == 0)
    assert sc[0] == exp["CI"]


@pytest.mark.parametrize("shape,seed", [((40, 36, 9), 1), ((70, 90, 12), 2), ((130, 104, 8), 3)])
def test_ci_vs_oracle_random_blobs(shape, seed):
    """Edge-touching and small arrays (s0 or s1 <= 100 exercises the duplicate-offset uniquing of
    np.intersect1d)."""
    rng = np.random.default_rng(seed)
    i, j, k = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
    d = np.zeros(shape, bool)
    for _ in range(7):
        c = [rng.uniform(-0.1, 1.1) * s for s in shape]
        r = rng.uniform(3, 12)
        d |= (i - c[0]) ** 2 + (j - c[1]) ** 2 + ((k - c[2]) * 3) ** 2 <= r * r
    d &= rng.random(shape) > 0.15
    vox = (1.5, 1.5, 10.0)
    table = compact_table(sphere_pix(vox, 50), shape)
    ref, _ = native.ci(d, table, vox)
    ci, sc, _ = _lib.ci(d, table, 1.5)
    assert np.array_equal(ci[0], ref)
    assert sc[0] == O.ci_scalar(ref[d])


def test_ci_errors():
    """Empty defect map -> IndexError (Vent_Analysis.py:270 / CI.py:118); a sphere that never drops
    below 50 % defect before the table's last radius -> ValueError (CI.py:101-103).  A radius-10
    table keeps offsets unaliased in a 40x40x24 all-defect volume, so interior voxels never stop."""
    table = compact_table(sphere_pix((1.5, 1.5, 10.0), 10), (40, 40, 24))
    with pytest.raises(IndexError):
        _lib.ci(np.zeros((40, 40, 24), np.uint8), table, 1.5)
    with pytest.raises(ValueError):
        _lib.ci(np.ones((40, 40, 24), np.uint8), table, 1.5)
    with pytest.raises(ValueError):
        native.ci(np.ones((40, 40, 24), np.uint8), table, (1.5, 1.5, 10.0))


def test_ci_table_api_equals_per_call_table():
    """vh_ci_tab with the HBM-resident table (vh_ci_table_create, reused across calls and batch
    sizes) equals vh_ci, which uploads the table per call; a table built for another (R, C) is
    refused; shells, maps and scalars bit-identical; shell=None skips that copy; a caller's own
    output array gets the same map."""
    import ctypes as ct
    rng = np.random.default_rng(5)
    shape = (70, 90, 12)
    i, j, k = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
    ds = []
    for _ in range(3):
        d = np.zeros(shape, bool)
        for _ in range(6):
            c = [rng.uniform(0, 1) * s for s in shape]
            r = rng.uniform(3, 10)
            d |= (i - c[0]) ** 2 + (j - c[1]) ** 2 + ((k - c[2]) * 3) ** 2 <= r * r
        ds.append(d.astype(np.uint8))
    vox = (1.5, 1.5, 10.0)
    table = compact_table(sphere_pix(vox, 50), shape)
    c = _lib.context(0)
    L = c.L
    for b in (1, 3):
        dd = np.ascontiguousarray(np.stack(ds[:b]))
        ci0 = np.empty(dd.shape, np.float64)
        sh0 = np.empty(dd.shape, np.int32)
        sc0 = np.zeros(b)
        c.check(L.vh_ci(c.h, _lib._ptr(dd), *shape, b, _lib._ptr(table.offsets), _lib._ptr(table.dup),
                        table.rows, _lib._ptr(table.bounds), _lib._ptr(table.radii),
                        table.bounds.shape[0], ct.c_double(1.5), _lib._ptr(ci0), _lib._ptr(sc0),
                        _lib._ptr(sh0)), "vh_ci")
        for _ in range(2):   # the second call reuses the device table
            ci1, sc1, sh1 = _lib.ci(dd, table, 1.5)
            assert np.array_equal(ci1, ci0) and np.array_equal(sc1, sc0) and np.array_equal(sh1, sh0)
        ci2, sc2, sh2 = _lib.ci(dd, table, 1.5, shell=False)
        assert sh2 is None and np.array_equal(ci2, ci0) and np.array_equal(sc2, sc0)
        # the map into a caller's pageable array (device map + copy) equals the device-mapped
        # pooled buffer the scatter writes directly
        ci3, sc3, _ = _lib.ci(dd, table, 1.5, shell=False, out=np.full(dd.shape, np.nan))
        assert np.array_equal(ci3, ci0) and np.array_equal(sc3, sc0)
        for q in range(b):
            ref, _ = native.ci(ds[q], table, vox)
            assert np.array_equal(ci0[q], ref)
    th = c.ci_table(table, shape[0], shape[1])
    other = np.zeros((60, 90, 12), np.uint8)
    other[30, 40, 5] = 1
    rc = L.vh_ci_tab(c.h, _lib._ptr(other), 60, 90, 12, 1, th, ct.c_double(1.5), None, None, None)
    assert rc == _lib.VH_ERR_ARG


def test_ci_threads_many_tables():
    """Several threads run CI on studies of 20 distinct voxel sizes (more than the 16 device
    tables a context keeps: evictions happen while other threads hold handles).  Every map equals
    the single-threaded oracle's (the table cache was unlocked, keyed by id())."""
    import threading
    from vent_analysis_amd import CI
    shape = (40, 36, 9)
    rng = np.random.default_rng(11)
    d = (rng.random(shape) < 0.2).astype(np.uint8)
    voxes = [(1.5, 1.5, 3.0 + 0.5 * i) for i in range(20)]
    refs = {}
    for vox in voxes:
        ref, _ = native.ci(d, compact_table(sphere_pix(vox, 12), shape), vox)
        refs[vox] = ref
    errors = []

    def worker(t):
        try:
            order = voxes[t:] + voxes[:t]
            for vox in order + order[::-1]:
                ci, _ = CI.calculate_CI_with_index(d, vox, Rmax=12)
                if not np.array_equal(ci, refs[vox]):
                    errors.append((t, vox))
        except Exception as e:   # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:4]
    c = _lib.context(0)
    assert len(c.ci_tables) <= c.CI_TABLES_KEPT


def ulps(a, b):
    """Distance in float32 units in the last place (same-sign values)."""
    ia = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(ia - ib)


def assert_n4_matches(out, its, conv, ref, its_ref, conv_ref, conv_mode, tag):
    """GPU N4 against the build-spec oracle (oracle/n4_oracle.c S1-S9).  U = L0 - B is bit-identical
    after every iteration, so the iteration counts and convergence values are identical; the output
    I / (float)exp((double)B) may differ by one float ulp only where OCML's and glibc's double exp
    round differently across a float midpoint (p ~ 2^-28 per voxel).  Tolerance: 1 ulp (north_star:
    1e-5 relative)."""
    assert list(its) == list(its_ref), (tag, list(its), list(its_ref))
    d = ulps(out, ref)
    assert d.max() <= 1, (tag, int(d.max()), int((d > 0).sum()))
    assert rel(out, ref) < 1e-5, tag
    if conv_mode == 0:   # float Welford: the same float recurrence over the same values
        assert np.array_equal(np.float32(conv), np.float32(conv_ref)), (tag, conv, conv_ref)
    else:                # exact CoV: double sums in a different order
        assert np.allclose(conv, conv_ref, rtol=1e-9), (tag, conv, conv_ref)


@pytest.mark.parametrize("conv_mode", [0, 1])
@pytest.mark.parametrize("shape,seed", [((64, 64, 16), 0), ((128, 128, 24), 0), ((96, 112, 20), 5),
                                        ((64, 64, 64), 6)])
def test_n4_vs_oracle(shape, seed, conv_mode):
    """Host entry point vh_n4 (one study: the per-iteration sweep driver)."""
    X, M = synth_volume(*shape, seed)
    ref, its_ref, conv_ref = native.n4(X, M, conv_mode=conv_mode)
    out, its, conv = _lib.n4(X, M.astype(np.uint8), conv_mode=conv_mode)
    assert np.all((its[0] >= 1) & (its[0] <= 50))
    assert_n4_matches(out[0], its[0], conv[0], ref, its_ref, conv_ref, conv_mode, (shape, seed))


def test_batch_pipeline_end_to_end():
    """Full calculate_VDP on a batch (N4 on device -> VDP chain), per-volume against the oracle
    applied to the GPU's N4 output (chain bit-exact) and the oracle N4 (tolerance)."""
    hp, mk = synth_batch(128, 128, 24, 3, base_seed=10)
    vox = (1.5, 1.5, 10.0)
    B = _lib.Batch(128, 128, 24, 3)
    B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=vox, do_cohort=True))
    n4, d, bo, lb, res = B.download(n4=True)
    for b in range(3):
        ref_n4, its_ref, _ = native.n4(hp[b], mk[b])
        assert list(res[b].n4_iters[:4]) == list(its_ref)
        assert rel(n4[b], ref_n4) < 1e-5
        o = O.calculate_vdp(n4[b], mk[b].astype(np.float64), vox, HP=hp[b])
        assert np.array_equal(d[b], o["defectArray"])
        assert np.array_equal(bo[b] == 1, o["defectBorder"])
        assert np.array_equal(lb[b], o["defectArrayLB"])
        assert res[b].vdp == o["VDP"]
        assert res[b].vdp_lb == o["VDP_lb"]
        assert res[b].n_km0 * 100 / mk[b].sum() == pytest.approx(o["VDP_km"], abs=0)
        assert rel(np.float32(res[b].snr), o["SNR"]) < 1e-5
    # cohort histogram = sum of per-volume float32 histograms
    h = B.cohort_hist()
    exp = np.zeros(_lib.COHORT_BINS, np.uint64)
    for b in range(3):
        nv = (n4[b] / np.float32(res[b].p99)).astype(np.float32)[mk[b] > 0]
        sel = (nv >= 0) & (nv < np.float32(1.5))
        bi = np.minimum((nv[sel] * np.float32(_lib.COHORT_BINS / 1.5)).astype(np.int64), 1023)
        exp += np.bincount(bi, minlength=_lib.COHORT_BINS).astype(np.uint64)
    assert np.array_equal(h, exp)
    B.close()


def test_rccl_cohort_allreduce_one_rank():
    """The RCCL path on one GPU (config 4's per-GPU shard): comm_unique_id -> comm_init(1, 0) ->
    a 256-volume 128x128x24 batch with the cohort histogram -> ncclAllReduce over one rank must
    leave the local histogram unchanged (api.hip vh_comm_init / vh_batch_cohort_allreduce)."""
    uid = _lib.comm_unique_id()
    assert len(uid) == _lib.COMM_ID_BYTES
    _lib.comm_init(1, 0, uid)
    try:
        assert _lib.comm_info() == (1, 0)   # RCCL's own rank count and rank (ncclCommCount)
        hp, mk = synth_batch(128, 128, 24, 256, base_seed=4000, unique=16)
        B = _lib.Batch(128, 128, 24, 256)
        B.upload(hp, mk)
        B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), do_cohort=True))
        local = B.cohort_hist()
        assert local.sum() > 0
        B.cohort_allreduce()
        B.sync()
        assert np.array_equal(B.cohort_hist(), local)
        B.close()
    finally:
        _lib.comm_destroy()


@pytest.mark.parametrize("shape,n,sub,slots,twos", [((64, 64, 16), 10, 4, 3, False),
                                                    ((64, 64, 16), 10, 4, 3, True),
                                                    ((128, 128, 24), 21, 8, 4, False),
                                                    ((37, 45, 7), 7, 3, 2, False),
                                                    ((37, 45, 7), 7, 3, 2, True)])
def test_pipe_host_to_host_equals_batch(shape, n, sub, slots, twos):
    """vh_pipe (slots x sub-volume sub-batches, ragged last sub-batch) returns exactly what one
    device-resident batch returns for the same studies: the mask crossing PCIe as bits (or as bytes
    when it holds values other than 0 / 1: twos), the output maps packed into one byte, the
    caller's whole pages pinned in place (the 128x128x24 case) and the chunk computes staggered."""
    R, C, Z = shape
    hp, mk = synth_batch(R, C, Z, n, base_seed=77)
    if twos:   # a mask value 2 somewhere outside the lung: the byte path must carry it as is
        mk = mk.copy()
        mk[:, 0, 0, :] = 2
    vox = (1.5, 1.5, 10.0)
    B = _lib.Batch(R, C, Z, n)
    B.upload(hp, mk)
    o = B.options(do_n4=True, vox=vox)
    B.run(o)
    ref = B.download(n4=True)
    B.close()
    P = _lib.Pipe(R, C, Z, sub, slots=slots)
    got = P.run(hp, mk, o)
    P.close()
    for a, b in zip(got[:4], ref[:4]):
        assert np.array_equal(a, b)
    for r, q in zip(got[4], ref[4]):   # (SNR is NaN for a study too small for its noise box)
        assert np.array_equal([r.vdp, r.vdp_lb, r.n_km0, r.snr] + list(r.n4_iters[:4]),
                              [q.vdp, q.vdp_lb, q.n_km0, q.snr] + list(q.n4_iters[:4]), equal_nan=True)


def test_pipe_pin_budget_stages_the_rest(monkeypatch):
    """VH_PIPE_PIN_CAP bounds the caller memory a run pins in place: past it the
    ranges go through the pinned staging, are counted (vh_pipe_stats) and the results are the same."""
    R, C, Z = 128, 128, 24
    n, sub, slots = 12, 4, 3
    hp, mk = synth_batch(R, C, Z, n, base_seed=91)
    o = _lib.Batch.options(do_n4=True, vox=(1.5, 1.5, 10.0))
    P = _lib.Pipe(R, C, Z, sub, slots=slots)
    ref = P.run(hp, mk, o)
    peak0, staged0 = P.stats()
    P.close()
    assert peak0 > 0 and staged0 == 0
    cap = 3 * sub * R * C * Z * 4   # about three chunks' inputs
    monkeypatch.setenv("VH_PIPE_PIN_CAP", str(cap))
    P = _lib.Pipe(R, C, Z, sub, slots=slots)
    got = P.run(hp, mk, o)
    peak, staged = P.stats()
    P.close()
    assert 0 < peak <= cap and staged > 0
    for a, b in zip(got[:4], ref[:4]):
        assert np.array_equal(a, b)


def test_batch_equals_single():
    hp, mk = synth_batch(64, 64, 16, 4, base_seed=3)
    B = _lib.Batch(64, 64, 16, 4)
    B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=(2, 2, 11.5)))
    n4, d, _, lb, res = B.download(n4=True)
    B.close()
    for b in range(4):
        out, its, _ = _lib.n4(hp[b], mk[b])
        assert np.array_equal(out[0], n4[b])
        assert list(its[0]) == list(res[b].n4_iters[:4])


def test_kmeans_vs_oracle():
    for seed in range(3):
        X, M = synth_volume(96, 96, 20, seed)
        _, _, _, res = _lib.vdp(X, M.astype(np.uint8), (1.5, 1.5, 10.0))
        sig = np.sort(X[M > 0])
        counts, centres, _ = O.kmeans_1d_sorted(sig)
        assert res[0].n_km0 == counts[0]
        assert np.allclose(list(res[0].km_centres), centres, rtol=1e-12)


def test_class_shim_matches_reference_goldens():
    from vent_analysis_amd import Vent_Analysis
    for path in GOLD:
        X, M, vox, exp, name = load_case(path)
        v = Vent_Analysis(xenon_array=X, mask_array=M, vox=vox)
        assert np.array_equal(v.mask_border, exp["mask_border"])
        v.N4_bias_correction = lambda H, Mk: H.astype(np.float32)   # as the goldens were made
        v.calculate_VDP()
        assert v.defectArray.dtype == np.float64 and v.defectArrayLB.dtype == np.float64
        assert np.array_equal(v.defectArray, exp["defect"])
        assert np.array_equal(v.defectBorder, exp["defect_border"])
        assert np.array_equal(v.defectArrayLB, exp["lb"])
        assert v.metadata["VDP"] == exp["VDP"]
        assert v.metadata["VDP_lb"] == exp["VDP_lb"]
        assert v.metadata["DefectVolume"] == exp["DefectVolume"]
        assert v.metadata["LungVolume"] == exp["LungVolume"]
        assert isinstance(v.metadata["SNR"], np.float32)
        assert rel(v.metadata["SNR"], exp["SNR"]) < 1e-5
        if "CI" in exp:
            v.calculate_CI()
            assert v.metadata["CI"] == exp["CI"]
            assert np.array_equal(v.CIarray[exp["defect"] > 0], exp["ci_values"])


def test_class_full_pipeline_with_n4():
    from vent_analysis_amd import Vent_Analysis
    X, M = synth_volume(128, 128, 24, 0)
    v = Vent_Analysis(xenon_array=X, mask_array=M, vox=(1.5, 1.5, 10.0))
    v.calculate_VDP()
    ref, its, _ = native.n4(X, M)
    assert v.N4HPvent.dtype == np.float32
    assert rel(v.N4HPvent, ref) < 1e-5
    o = O.calculate_vdp(v.N4HPvent, M, (1.5, 1.5, 10.0), HP=X)
    assert v.metadata["VDP"] == o["VDP"]
    n4b = v.N4_bias_correction(X, M)
    assert np.array_equal(n4b, v.N4HPvent)



@pytest.mark.parametrize("v", [255, 2])
def test_class_single_value_mask_vs_reference(v):
    """A 0/v mask (mask DICOM folders often hold 0/255): with N4 := identity, as the
    goldens were made, the class gives the reference's expressions on the v-scaled maps
    (oracle.calculate_vdp_literal: scipy's medfilt2d on (mn < thresh) * mask, LB * mask) and the
    golden VDP / SNR / CI."""
    from vent_analysis_amd import Vent_Analysis
    for path in GOLD:
        X, M, vox, exp, name = load_case(path)
        Mv = M * v
        va = Vent_Analysis(xenon_array=X, mask_array=Mv, vox=vox)
        va.N4_bias_correction = lambda H, Mk: H.astype(np.float32)
        va.calculate_VDP()
        o = O.calculate_vdp_literal(X, Mv, vox)
        assert va.defectArray.dtype == np.float64 and va.defectArrayLB.dtype == np.float64, name
        assert np.array_equal(va.defectArray, o["defectArray"]), name
        assert np.array_equal(va.defectArray, exp["defect"] * np.float64(v)), name
        assert np.array_equal(va.defectBorder, exp["defect_border"]), name
        assert np.array_equal(va.defectArrayLB, o["defectArrayLB"]), name
        for k in ("VDP", "VDP_lb", "DefectVolume"):
            assert va.metadata[k] == o[k], (name, k)
        assert va.metadata["VDP"] == exp["VDP"], name
        assert va.metadata["LungVolume"] == 0.0   # np.sum(mask == 1) (:166)
        assert rel(va.metadata["SNR"], exp["SNR"]) < 1e-5
        if "CI" in exp:
            va.calculate_CI()
            assert va.metadata["CI"] == exp["CI"]
            assert np.array_equal(va.CIarray[exp["defect"] > 0], exp["ci_values"])


def test_class_255_mask_full_pipeline():
    """Without an N4 override: a 0/255 mask has no voxel of SimpleITK N4's label 1 (the mask is
    cast to UInt8, MaskLabel 1), so N4HPvent is HPvent itself (parity unpinned, see
    Vent_Analysis.calculate_VDP) and the chain equals the literal oracle on it."""
    from vent_analysis_amd import Vent_Analysis
    X, M = synth_volume(128, 128, 24, 0)
    va = Vent_Analysis(xenon_array=X, mask_array=M * 255.0, vox=(1.5, 1.5, 10.0))
    va.calculate_VDP()
    assert va.N4HPvent.dtype == np.float32 and np.array_equal(va.N4HPvent, X)
    assert va.n4_iterations == [0, 0, 0, 0]
    o = O.calculate_vdp_literal(X, M * 255.0, (1.5, 1.5, 10.0))
    assert np.array_equal(va.defectArray, o["defectArray"])
    assert np.array_equal(va.defectArrayLB, o["defectArrayLB"])
    for k in ("VDP", "VDP_lb", "DefectVolume"):
        assert va.metadata[k] == o[k], k
    assert va.metadata["VDP_lb"] == 0.0 and va.metadata["DefectVolume"] == 0.0
    assert rel(va.metadata["SNR"], O.calculate_snr(X, M)) < 1e-5
    assert np.array_equal(va.N4_bias_correction(X, M * 255.0), X)
    with pytest.raises(ValueError):   # several nonzero values: a median over mixed values
        Vent_Analysis(xenon_array=X, mask_array=M * (1 + (np.arange(M.shape[2]) % 2)),
                      vox=(1.5, 1.5, 10.0)).calculate_VDP()


def test_pickle_and_nifti_of_gpu_study(tmp_path):
    """SURVEY 8(f) rank 2 on device outputs: a GPU-computed study (calculate_VDP with N4 +
    calculate_CI) through pickleMe -> Vent_Analysis(pickle_path=) keeps every array bit for bit
    with the reference's dtypes (defectArray f64, defectBorder bool, defectArrayLB
    f64, CIarray f64, N4HPvent f32, SNR f32), and exportNifti's six channels are those arrays
    (Vent_Analysis.py:273-313, 542-559)."""
    from vent_analysis_amd import Vent_Analysis, nifti
    X, M = synth_volume(128, 128, 24, 0)
    P = (X * 0.5 + 3).astype(np.float32)
    va = Vent_Analysis(xenon_array=X, mask_array=M, proton_array=P, vox=(1.5, 1.5, 10.0))
    va.calculate_VDP()
    va.calculate_CI()
    va.metadata["PatientName"] = "Test^Pickle"
    pk = str(tmp_path / "study.pkl")
    va.pickleMe(pk)
    vb = Vent_Analysis(pickle_path=pk)
    dtypes = {"defectArray": np.float64, "defectBorder": np.bool_, "defectArrayLB": np.float64,
              "CIarray": np.float64, "N4HPvent": np.float32, "mask_border": np.float64}
    for k, dt in dtypes.items():
        a, b = getattr(va, k), getattr(vb, k)
        assert b.dtype == dt, (k, b.dtype)
        assert np.array_equal(a, b), k
    for k in ("HPvent", "mask", "proton"):
        assert np.array_equal(getattr(va, k), getattr(vb, k)), k
    assert isinstance(vb.metadata["SNR"], np.float32)
    for k, val in va.metadata.items():
        assert vb.metadata[k] == val or (val != val and vb.metadata[k] != vb.metadata[k]), k
    assert vb.vox == va.vox and vb.version == va.version
    o = O.calculate_vdp(vb.N4HPvent, M, (1.5, 1.5, 10.0), HP=X)
    assert np.array_equal(vb.defectArray, o["defectArray"]) and vb.metadata["VDP"] == o["VDP"]
    vb.exportNifti(str(tmp_path), "study")
    data, _, _ = nifti.load(str(tmp_path / "study_dataArray.nii"))
    assert data.shape == X.shape + (6,) and data.dtype == np.float32
    for ch, a in enumerate((P, X, M, vb.N4HPvent, vb.defectArray, vb.CIarray)):
        assert np.array_equal(data[..., ch], np.asarray(a, np.float32)), ch

# ---- ragged / degenerate shapes and full-size properties -------------------------------------
RAGGED = [((37, 45, 7), 11), ((12, 70, 9), 12), ((12, 70, 9), 13), ((130, 20, 3), 13),
          ((5, 90, 12), 14), ((70, 5, 30), 15), ((66, 66, 2), 16), ((129, 33, 5), 17),
          ((40, 40, 40), 18), ((31, 97, 11), 19), ((64, 65, 4), 20), ((65, 64, 17), 21),
          ((100, 30, 23), 22), ((23, 100, 3), 23), ((48, 48, 9), 24), ((80, 24, 24), 25),
          ((17, 17, 17), 26), ((90, 110, 6), 27), ((127, 61, 8), 28), ((33, 128, 13), 29)]


@pytest.mark.parametrize("conv_mode", [0, 1])
@pytest.mark.parametrize("driver", ["sweep", "study", "grid"])
@pytest.mark.parametrize("shape,seed", RAGGED, ids=lambda v: "x".join(map(str, v)) if isinstance(v, tuple) else str(v))
def test_n4_ragged_shapes_vs_oracle(shape, seed, driver, conv_mode):
    """Rows past one 64-row slot, columns not a multiple of the 64-column tile, 2- and 3-slice
    volumes, single-row-slot studies, masks touching the borders; both drivers, both convergence
    measures.  (12x70x9 seed 13 is the round-1 case whose 1-ulp U differences flipped ITK's bin
    minimum; with both sides evaluating S1-S9 it matches like every other case.)"""
    X, M = synth_volume(*shape, seed)
    if M.sum() < 4:
        pytest.skip("mask too small for the generator at this shape")
    ref, its_ref, conv_ref = native.n4(X, M, conv_mode=conv_mode)
    try:
        n4, d, _, lb, res = _run_batch(X[None], M.astype(np.uint8)[None], driver, conv_mode=conv_mode)
    except ValueError as e:   # the study driver holds a study's state in LDS: not every shape fits
        if driver in ("study", "grid") and "LDS budget" in str(e):
            pytest.skip(str(e))
        raise
    assert_n4_matches(n4[0], res[0].n4_iters[:4], res[0].n4_conv[:4], ref, its_ref, conv_ref,
                      conv_mode, (shape, seed, driver))


def _single_slice(R, C, seed):
    rng = np.random.default_rng(seed)
    i, j = np.meshgrid(np.arange(R), np.arange(C), indexing="ij")
    m = (((i - R / 2) / (0.4 * R)) ** 2 + ((j - C / 2) / (0.3 * C)) ** 2) <= 1
    x = (np.where(m, 150.0, 0.0) * np.exp(0.3 * i / R) + rng.rayleigh(10, m.shape))
    x[m & (rng.random(m.shape) < 0.15)] *= 0.2
    return x.astype(np.float32)[:, :, None], m.astype(np.float64)[:, :, None]


@pytest.mark.parametrize("case", ["37x45x7", "50x33x1", "19x130x5", "64x200x1"])
def test_vdp_chain_ragged_vs_oracle(case):
    R, C, Z = (int(v) for v in case.split("x"))
    if Z == 1:
        X, M = _single_slice(R, C, R + C)
    else:
        X, M = synth_volume(R, C, Z, R + C + Z)
    vox = (1.5, 1.5, 10.0)
    d, bo, lb, res = _lib.vdp(X, M.astype(np.uint8), vox)
    o = O.calculate_vdp(X, M, vox, HP=X)
    assert np.array_equal(d[0], o["defectArray"])
    assert np.array_equal(bo[0] == 1, o["defectBorder"])
    assert np.array_equal(lb[0], o["defectArrayLB"])
    assert res[0].vdp == o["VDP"] and res[0].vdp_lb == o["VDP_lb"]
    assert np.float32(res[0].mean_anchor) == o["mean_anchor"] and np.float32(res[0].p99) == o["p99"]
    assert np.array_equal(_lib.border(M.astype(np.uint8))[0], O.calculate_border(M))


@pytest.mark.parametrize("shape", [(256, 256, 64), (160, 200, 140)])
def test_large_single_volume_grid_sort_vs_oracle(shape):
    """One volume of >= 2^22 voxels takes the grid radix sort (k_sortg_*, 4 passes over 8192-key
    chunks) and the wave-parallel k-means tile sums: the sorted-key statistics (numpy-order mean,
    p99 order statistic) and the maps equal the oracle bit for bit; the k-means partition matches
    the oracle's Lloyd run on the sorted values."""
    X, M = synth_volume(*shape, 41)
    vox = (1.0, 1.0, 1.0)
    d, bo, lb, res = _lib.vdp(X, M.astype(np.uint8), vox)
    o = O.calculate_vdp(X, M, vox, HP=X)
    assert np.float32(res[0].mean_anchor) == o["mean_anchor"] and np.float32(res[0].p99) == o["p99"]
    assert np.array_equal(d[0], o["defectArray"]) and np.array_equal(lb[0], o["defectArrayLB"])
    assert res[0].vdp == o["VDP"] and res[0].vdp_lb == o["VDP_lb"]
    s = np.sort(X[M > 0].astype(np.float32))
    counts, centres, _ = O.kmeans_1d_sorted(s)
    assert int(res[0].n_km0) == int(counts[0])
    assert np.allclose(list(res[0].km_centres), centres, rtol=1e-12)


def test_kmeans_global_tile_prefix_vs_oracle():
    """A volume with more than 4096 k-means tiles (> 4.19 M masked voxels) takes the multi-workgroup
    tile sums (k_km_tiles) and the global-memory prefix of k_kmeans: partition and centres against the
    oracle's Lloyd run on the sorted values; the sorted-list statistics bit-exact."""
    X, M = synth_volume(336, 336, 192, 43)
    assert (M > 0).sum() > 4096 * 1024
    d, bo, lb, res = _lib.vdp(X, M.astype(np.uint8), (1.0, 1.0, 1.0))
    s = np.sort(X[M > 0].astype(np.float32))
    counts, centres, _ = O.kmeans_1d_sorted(s)
    assert int(res[0].n_km0) == int(counts[0])
    assert np.allclose(list(res[0].km_centres), centres, rtol=1e-12)
    assert np.float32(res[0].p99) == s[int(len(s) * 0.99)]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 64, 65, 127, 129, 4095, 4097, 262143, 262144, 262145,
                               300000])
def test_kmeans_one_wave_kernel_sizes(n, monkeypatch):
    """k_kmeans_s (volumes of up to 2^19 voxels) at masked counts around its 64-key tiles, its
    192-key windows and its sample stride (one sample per tile up to 2^18 keys, per two tiles above):
    the partition and the centres against the oracle's Lloyd run, and against the multi-wave
    k_kmeans on the same data (VH_KM_OLD=1)."""
    R, C, Z = 128, 128, 32   # V = 2^19
    rng = np.random.default_rng(1000 + n)
    X = (rng.gamma(4.0, 50.0, size=(R, C, Z)) + 1.0).astype(np.float32)
    M = np.zeros(R * C * Z, np.uint8)
    M[rng.choice(R * C * Z, n, replace=False)] = 1
    M = M.reshape(R, C, Z)
    vox = (1.5, 1.5, 10.0)
    res = _lib.vdp(X, M, vox)[3]
    counts, centres, _ = O.kmeans_1d_sorted(np.sort(X[M > 0]))
    assert int(res[0].n_km0) == O.kmeans_low_count(counts)
    assert np.allclose(list(res[0].km_centres), centres, rtol=1e-12)
    monkeypatch.setenv("VH_KM_OLD", "1")
    old = _lib.vdp(X, M, vox)[3]
    assert int(old[0].n_km0) == int(res[0].n_km0)
    assert np.allclose(list(old[0].km_centres), list(res[0].km_centres), rtol=1e-12)


def test_empty_mask_volume_in_batch():
    """A study with an empty mask must not disturb its neighbours; the class raises IndexError
    like the reference's sorted-list indexing (Vent_Analysis.py:255)."""
    hp, mk = synth_batch(64, 64, 16, 3, base_seed=7)
    mk[1] = 0
    B = _lib.Batch(64, 64, 16, 3)
    B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0)))
    n4, d, _, _, res = B.download(n4=True)
    B.close()
    assert res[1].n_mask == 0 and d[1].sum() == 0
    assert np.array_equal(n4[1], hp[1])                  # B = 0: I / exp(0)
    for b in (0, 2):
        out, its, _ = _lib.n4(hp[b], mk[b])
        assert np.array_equal(out[0], n4[b])
        assert list(its[0]) == list(res[b].n4_iters[:4])
    from vent_analysis_amd import Vent_Analysis
    v = Vent_Analysis(xenon_array=hp[1], mask_array=np.zeros((64, 64, 16)), vox=(1.5, 1.5, 10.0))
    with pytest.raises(IndexError):
        v.calculate_VDP()


def test_full_size_batch_properties():
    """bench configuration (256 x 128x128x24, 16 distinct studies repeated): size-independent
    properties -- counts match the maps, defects lie in the mask, repeated studies give identical
    results wherever they sit in the batch, a second run is identical, and the cohort histogram
    equals the numpy histogram of the p99-normalised masked N4 values."""
    nb = 256
    hp, mk = synth_batch(128, 128, 24, nb, base_seed=0, unique=16)
    B = _lib.Batch(128, 128, 24, nb)
    B.upload(hp, mk)
    o = B.options(do_n4=True, vox=(1.5, 1.5, 10.0), do_cohort=True)
    B.run(o)
    n4, d, bo, lb, res = B.download(n4=True)
    h1 = B.cohort_hist()
    B.run(o)
    n4b, d2, _, lb2, res2 = B.download(n4=True)
    B.close()
    assert np.array_equal(n4, n4b) and np.array_equal(d, d2) and np.array_equal(lb, lb2)
    for b in range(nb):
        r = res[b]
        assert r.n_defect == int(d[b].sum())
        assert r.n_lb12 == int(((lb[b] == 1) | (lb[b] == 2)).sum())
        assert not np.any(d[b] & (mk[b] == 0))
        assert r.n_mask == int((mk[b] > 0).sum())
        assert all(1 <= k <= 50 for k in r.n4_iters[:4])
        assert r.vdp == res2[b].vdp
        if b >= 16:
            assert np.array_equal(n4[b], n4[b % 16]) and r.vdp == res[b % 16].vdp
    exp = np.zeros(_lib.COHORT_BINS, np.uint64)
    for b in range(nb):
        nv = (n4[b] / np.float32(res[b].p99)).astype(np.float32)[mk[b] > 0]
        sel = (nv >= 0) & (nv < np.float32(1.5))
        bi = np.minimum((nv[sel] * np.float32(_lib.COHORT_BINS / 1.5)).astype(np.int64), 1023)
        exp += np.bincount(bi, minlength=_lib.COHORT_BINS).astype(np.uint64)
    assert np.array_equal(h1, exp)


def test_bench_workload_vs_oracle():
    """The exact batch bench.py times at N=1 (256 x 128x128x24, 64 distinct studies with per-study
    lung geometry, masked voxels +-20 %: synth_batch(..., unique=64, vary=True)) through the default
    path (k_n4_study with PC).  Every distinct study against the C oracle: per-level iterations,
    identical float32 convergence values, N4HPvent within 1 ulp; the post-N4 chain bit-exact against
    the numpy oracle applied to the GPU's N4HPvent; the repeated studies identical to their first
    copy wherever they sit in the batch."""
    import bench
    from concurrent.futures import ThreadPoolExecutor
    nb, R, C, Z = 256, 128, 128, 24
    vox = (1.5, 1.5, 10.0)
    hp, mk = synth_batch(R, C, Z, nb, base_seed=bench.shard_seed(0), unique=bench.BENCH_UNIQUE,
                         vary=True)
    B = _lib.Batch(R, C, Z, nb)
    B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=vox, do_cohort=True))
    n4, d, bo, lb, res = B.download(n4=True)
    B.close()
    u = bench.BENCH_UNIQUE
    for b in range(u, nb):
        assert np.array_equal(n4[b], n4[b % u]) and np.array_equal(d[b], d[b % u])
        assert list(res[b].n4_iters[:4]) == list(res[b % u].n4_iters[:4])
    with ThreadPoolExecutor(16) as ex:   # ctypes drops the GIL: the oracle runs in parallel
        refs = list(ex.map(lambda b: native.n4(hp[b], mk[b]), range(u)))
    nmask = [int((mk[b] == 1).sum()) for b in range(u)]
    assert max(nmask) > 1.15 * min(nmask)   # the heterogeneous batch, not 64 copies of one geometry
    for b in range(u):
        ref, its_ref, conv_ref = refs[b]
        assert_n4_matches(n4[b], res[b].n4_iters[:4], res[b].n4_conv[:4], ref, its_ref, conv_ref,
                          0, ("bench", b))
        o = O.calculate_vdp(n4[b], mk[b].astype(np.float64), vox, HP=hp[b])
        assert np.array_equal(d[b], o["defectArray"]), b
        assert np.array_equal(bo[b] == 1, o["defectBorder"]), b
        assert np.array_equal(lb[b], o["defectArrayLB"]), b
        assert res[b].vdp == o["VDP"] and res[b].vdp_lb == o["VDP_lb"], b
        assert np.float32(res[b].mean_anchor) == o["mean_anchor"], b
        assert np.float32(res[b].p99) == o["p99"], b
        assert res[b].n_km0 * 100 / mk[b].sum() == pytest.approx(o["VDP_km"], abs=0), b
        assert rel(np.float32(res[b].snr), o["SNR"]) < 1e-5, b


# ---- BASELINE configs 2 and 5 --------------------------------------------------------------------
@pytest.mark.parametrize("shape,seed", [((64, 64, 16), 0), ((37, 45, 7), 3), ((48, 48, 48), 4)])
def test_vdp_chain_morph3d_vs_oracle(shape, seed):
    """Build-defined 3-D morphology (config 5): 3x3x3 majority + 3-axis np.gradient border."""
    hp, mk = synth_batch(*shape, 2, base_seed=seed)
    vox = (1.0, 1.0, 1.0)
    B = _lib.Batch(*shape, 2)
    B.upload(hp, mk)
    B.run(B.options(do_n4=False, vox=vox, morph3d=True))
    _, d, bo, lb, res = B.download()
    B.close()
    for b in range(2):
        o = O.calculate_vdp(hp[b], mk[b].astype(np.float64), vox, HP=hp[b], morph3d=True)
        assert np.array_equal(d[b], o["defectArray"])
        assert np.array_equal(bo[b] == 1, o["defectBorder"])
        assert np.array_equal(lb[b], o["defectArrayLB"])
        assert res[b].vdp == o["VDP"]


@pytest.mark.parametrize("shape,m3d", [((37, 45, 7), False), ((20, 300, 16), False),
                                        ((10, 150, 30), False), ((33, 70, 13), True),
                                        ((12, 90, 64), True), ((5, 8, 1), False)])
def test_plane_sweep_equals_tile_kernel_and_oracle(shape, m3d, monkeypatch):
    """classify / border: the plane-sweep kernel (default) against the halo-tile kernel
    (VH_CLASSIFY_TILE=1) and the oracle, on dense random masks (many median flips), Z % 4 != 0
    and planes split into column bands (C * ceil(Z / 4) > 1024 words)."""
    rng = np.random.default_rng(sum(shape))
    hp = rng.rayleigh(10.0, (2,) + shape).astype(np.float32) + 1.0
    mk = (rng.random((2,) + shape) < 0.7).astype(np.uint8)
    vox = (1.0, 1.0, 1.0)

    def run():
        B = _lib.Batch(*shape, 2)
        B.upload(hp, mk)
        B.run(B.options(do_n4=False, vox=vox, morph3d=m3d, do_snr=False))
        out = B.download()
        B.close()
        return out, _lib.border(mk)

    (_, d, bo, lb, res), mb = run()
    monkeypatch.setenv("VH_CLASSIFY_TILE", "1")
    (_, d2, bo2, lb2, res2), mb2 = run()
    assert np.array_equal(d, d2) and np.array_equal(bo, bo2) and np.array_equal(lb, lb2)
    assert np.array_equal(mb, mb2)
    for b in range(2):
        assert res[b].n_defect == res2[b].n_defect == int(d[b].sum())
        assert res[b].n_lb12 == res2[b].n_lb12
        o = O.calculate_vdp(hp[b], mk[b].astype(np.float64), vox, HP=hp[b], morph3d=m3d)
        assert np.array_equal(d[b], o["defectArray"])
        assert np.array_equal(bo[b] == 1, o["defectBorder"])
        assert np.array_equal(lb[b], o["defectArrayLB"])
    assert np.array_equal(mb[0], O.calculate_border(mk[0].astype(np.float64)))


def test_config2_256x256x24_full_pipeline_vs_oracle():
    """Config 2: one 256x256x24 study, N4 + normalise + mean-anchored VDP."""
    X, M = synth_volume(256, 256, 24, 7)
    vox = (1.5, 1.5, 10.0)
    B = _lib.Batch(256, 256, 24, 1)
    B.upload(X[None], M.astype(np.uint8)[None])
    B.run(B.options(do_n4=True, vox=vox))
    n4, d, bo, lb, res = B.download(n4=True)
    B.close()
    ref, its, _ = native.n4(X, M)
    assert list(res[0].n4_iters[:4]) == list(its)
    assert rel(n4[0], ref) < 1e-5
    o = O.calculate_vdp(n4[0], M, vox, HP=X)
    assert np.array_equal(d[0], o["defectArray"]) and res[0].vdp == o["VDP"]
    assert np.array_equal(lb[0], o["defectArrayLB"]) and res[0].vdp_lb == o["VDP_lb"]


def test_config5_512_cubed_n4_morph3d():
    """Config 5: one 512^3 isotropic study, N4 multiresolution + 3-D morphology.  N4 is pinned by
    tests/golden/n4_512_seed11.npz (scripts/make_n4_512_fixture.py ran the C oracle once in the
    build container): per-level iterations and convergence values, a strided voxel sample and the
    sha256 of the whole N4HPvent; plus run-to-run determinism.  The post-N4 chain is checked
    bit-exactly against the oracle applied to the GPU's N4 output."""
    n = 512
    X, M = synth_volume(n, n, n, 11)
    vox = (1.0, 1.0, 1.0)
    B = _lib.Batch(n, n, n, 1)
    B.upload(X[None], M.astype(np.uint8)[None])
    o = B.options(do_n4=True, vox=vox, morph3d=True)
    B.run(o)
    n4, d, bo, lb, res = B.download(n4=True)
    B.run(o)
    n4b, _, _, _, res2 = B.download(n4=True, maps=False)
    B.close()
    assert np.array_equal(n4[0], n4b[0]) and list(res[0].n4_iters) == list(res2[0].n4_iters)
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "n4_512_seed11.npz"))
    assert list(res[0].n4_iters[:4]) == fx["iters"].tolist()
    assert np.array_equal(np.float32(res[0].n4_conv[:4]), fx["conv"])
    flat = n4[0].reshape(-1)
    assert rel(flat[fx["sample_idx"]], fx["sample_val"]) < 1e-5
    assert hashlib.sha256(np.ascontiguousarray(n4[0]).tobytes()).hexdigest() == str(fx["sha256"])
    assert np.all(np.isfinite(n4[0])) and np.all((n4[0] > 0) == (X > 0))
    ref = O.calculate_vdp(n4[0], M, vox, morph3d=True)
    assert np.array_equal(d[0], ref["defectArray"])
    assert np.array_equal(bo[0] == 1, ref["defectBorder"])
    assert res[0].vdp == ref["VDP"] and res[0].vdp_lb == ref["VDP_lb"]


@pytest.mark.parametrize("shape", [(256, 256, 256), (192, 160, 96)])
def test_n4_sweep_rerun_bit_identical(shape):
    """Re-running one batch gives bit-identical fields, iteration counts and convergence values
    (the sweep driver's multi-workgroup eval once scattered the convergence input across lines
    shared by workgroups; 256^3 lost ~1e4 values per iteration run-to-run)."""
    X, M = synth_volume(*shape, 11)
    B = _lib.Batch(*shape, 1)
    B.upload(X[None], M.astype(np.uint8)[None])
    o = B.options(do_n4=True, vox=(1.0, 1.0, 1.0), n4_mode="sweep", do_snr=False, do_kmeans=False)
    outs = []
    for _ in range(3):
        B.run(o)
        n4, _, _, _, res = B.download(n4=True, maps=False)
        outs.append((n4[0].copy(), list(res[0].n4_iters[:4]), [float(c) for c in res[0].n4_conv[:4]]))
    B.close()
    for n4, its, conv in outs[1:]:
        assert its == outs[0][1] and conv == outs[0][2]
        assert np.array_equal(n4, outs[0][0])


@pytest.mark.parametrize("shape,grid", [((96, 112, 20), "0"), ((256, 256, 24), "1"), ((128, 128, 96), "1")])
def test_n4_pc_equals_serial_chain(shape, grid, monkeypatch):
    """S7 by guess and verify (k_n4_pcw one workgroup, k_n4_pcg the cooperative grid for one large
    volume) against the serial float Welford chain (VH_N4_SERIAL_CHAIN) on the sweep driver: the same
    iteration counts, the same convergence values and the same field, bit for bit."""
    X, M = synth_volume(*shape, 31)
    outs = []
    for serial in (False, True):
        if serial:
            monkeypatch.setenv("VH_N4_SERIAL_CHAIN", "1")
        else:
            monkeypatch.delenv("VH_N4_SERIAL_CHAIN", raising=False)
        monkeypatch.setenv("VH_N4_PCG", grid)
        B = _lib.Batch(*shape, 1)
        B.upload(X[None], M.astype(np.uint8)[None])
        B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode="sweep", do_snr=False, do_kmeans=False))
        n4, _, _, _, res = B.download(n4=True, maps=False)
        B.close()
        outs.append((n4[0].copy(), list(res[0].n4_iters[:4]), [float(c) for c in res[0].n4_conv[:4]]))
    assert outs[0][1] == outs[1][1] and outs[0][2] == outs[1][2]
    assert np.array_equal(outs[0][0], outs[1][0])


# ---- volume-resident N4 driver (one workgroup per study) ------------------------------------------
def _run_batch(hp, mk, mode, **kw):
    R, C, Z = hp.shape[1:]
    B = _lib.Batch(R, C, Z, hp.shape[0])
    B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=mode, **kw))
    out = B.download(n4=True)
    B.close()
    return out


@pytest.mark.parametrize("conv_mode", [0, 1])
@pytest.mark.parametrize("shape,nb,seed", [((128, 128, 24), 3, 0), ((96, 112, 20), 2, 5),
                                           ((64, 64, 32), 2, 6), ((37, 45, 7), 2, 11),
                                           ((12, 70, 9), 2, 12), ((130, 20, 3), 2, 13)])
def test_n4_study_vs_oracle(shape, nb, seed, conv_mode):
    """n4_mode=2 (k_n4_study), several studies per launch, against the C oracle."""
    hp, mk = synth_batch(*shape, nb, base_seed=seed)
    n4, d, _, lb, res = _run_batch(hp, mk, "study", conv_mode=conv_mode)
    for b in range(nb):
        ref, its_ref, conv_ref = native.n4(hp[b], mk[b], conv_mode=conv_mode)
        assert_n4_matches(n4[b], res[b].n4_iters[:4], res[b].n4_conv[:4], ref, its_ref, conv_ref,
                          conv_mode, (shape, seed, b))


def test_n4_study_deterministic_and_equal_to_sweeps():
    """Both drivers evaluate S1-S9 operation for operation: identical outputs, not just close."""
    hp, mk = synth_batch(128, 128, 24, 4, base_seed=20)
    a = _run_batch(hp, mk, "study")
    b = _run_batch(hp, mk, "study")
    s = _run_batch(hp, mk, "sweep")
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert np.array_equal(a[0], s[0]) and np.array_equal(a[1], s[1])
    for v in range(4):
        assert list(a[4][v].n4_iters[:4]) == list(s[4][v].n4_iters[:4])
        assert a[4][v].n4_conv[:4] == s[4][v].n4_conv[:4]


def test_n4_study_empty_mask_in_batch():
    hp, mk = synth_batch(64, 64, 16, 3, base_seed=7)
    mk[1] = 0
    n4, d, _, _, res = _run_batch(hp, mk, "study")
    assert res[1].n_mask == 0 and d[1].sum() == 0
    assert np.array_equal(n4[1], hp[1])
    for b in (0, 2):
        ref, its, _ = native.n4(hp[b], mk[b])
        assert list(its) == list(res[b].n4_iters[:4])
        assert rel(n4[b], ref) < 1e-5


# ---- sorted-list statistics on adversarial value distributions ------------------------------------
def test_mean_anchor_partial_chunk_lengths():
    """k_chunk_sums: numpy's pairwise tree of the last, partial 8192-chunk of each volume (built
    level by level in LDS) for masked counts around every leaf / split edge (< 8, 8, 128, 129,
    130, 255, 256, 1000, 8191, 8192, 8193, 16385, 33000): mean anchor bit-exact to np.mean of the
    sorted list (oracle mean_f32, pinned to numpy)."""
    rng = np.random.default_rng(11)
    shape = (64, 64, 12)
    counts = [1, 5, 8, 9, 127, 128, 129, 130, 255, 256, 1000, 4097, 8191, 8192, 8193, 16385, 33000,
              49151]
    B = _lib.Batch(*shape, len(counts))
    X = np.zeros((len(counts),) + shape, np.float32)
    M = np.zeros((len(counts),) + shape, np.uint8)
    for b, n in enumerate(counts):
        idx = rng.choice(X[b].size, n, replace=False)
        M[b].flat[idx] = 1
        X[b].flat[idx] = (rng.gamma(2.0, 50.0, n) + 1).astype(np.float32)
    B.upload(X, M)
    B.run(B.options(do_n4=False, vox=(1.5, 1.5, 10.0)))
    _, _, _, _, res = B.download(maps=False)
    B.close()
    for b, n in enumerate(counts):
        s_ = np.sort(X[b][M[b] > 0])
        assert np.float32(res[b].mean_anchor) == O.mean_f32(s_) == np.mean(s_), n
        assert np.float32(res[b].p99) == s_[int(n * 0.99)], n


@pytest.mark.parametrize("kind", ["constant", "two_values", "three_values", "negative", "ulp_range",
                                  "decades"])
def test_sorted_statistics_adversarial(kind):
    """The per-volume radix sort (k_sort_vol), the numpy-order mean anchor, p99, k-means and the
    cohort rows on value distributions the synthetic generator never makes: a single value (every
    digit of every key in one bin: the histogram's one-add path), two values (degenerate k-means
    centres), mostly negative values (sign-flipped keys; p99 < 0 takes the cohort scan path), a
    4-ulp range (only the low digit varies), 8 decades.  N4 := identity; two volumes per batch,
    the second the first flipped, so two segments of the batch are exercised."""
    rng = np.random.default_rng(7)
    shape = (48, 40, 12)
    M = (rng.random(shape) < 0.6).astype(np.uint8)
    n = int(M.sum())
    if kind == "constant":
        v = np.full(n, 3.25, np.float32)
    elif kind == "two_values":
        v = rng.choice(np.float32([1.5, 2.5]), n)
    elif kind == "three_values":   # 5 % / 15 % / 80 %: equal initial centres, a mixed first cluster
        v = rng.choice(np.float32([1.0, 2.0, 10.0]), n, p=[0.05, 0.15, 0.8])
    elif kind == "negative":
        v = rng.normal(-150.0, 50.0, n).astype(np.float32)
    elif kind == "ulp_range":
        v = np.float32(100) + rng.integers(0, 4, n).astype(np.float32) * np.spacing(np.float32(100))
    else:
        v = (10.0 ** rng.uniform(-4, 4, n)).astype(np.float32)
    X = np.zeros(shape, np.float32)
    X[M == 1] = v
    vols = [(X, M), (np.ascontiguousarray(X[::-1]), np.ascontiguousarray(M[::-1]))]
    B = _lib.Batch(*shape, 2)
    B.upload(np.stack([a for a, _ in vols]), np.stack([m for _, m in vols]))
    B.run(B.options(do_n4=False, vox=(1.5, 1.5, 10.0), do_cohort=True))
    _, d, _, lb, res = B.download()
    h = B.cohort_hist()
    B.close()
    exp_h = np.zeros(_lib.COHORT_BINS, np.uint64)
    for b, (XX, MM) in enumerate(vols):
        o = O.calculate_vdp(XX, MM.astype(np.float64), (1.5, 1.5, 10.0))
        assert np.float32(res[b].mean_anchor) == o["mean_anchor"]
        assert np.float32(res[b].p99) == o["p99"]
        assert np.array_equal(d[b], o["defectArray"])
        assert np.array_equal(lb[b], o["defectArrayLB"])
        # degenerate inputs included: empty clusters take the farthest value
        # (oracle kmeans_1d_sorted, pinned to scikit-learn in tests/test_kmeans_oracle.py)
        assert res[b].n_km0 * 100 / MM.sum() == pytest.approx(o["VDP_km"], abs=0)
        assert np.allclose(list(res[b].km_centres), o["km_centres"], rtol=1e-12, atol=0)
        if kind in ("two_values", "three_values"):   # every value a cluster of its own
            assert res[b].n_km0 == int((XX[MM > 0] == XX[MM > 0].min()).sum())
        nv = (XX / np.float32(res[b].p99)).astype(np.float32)[MM > 0]
        sel = (nv >= 0) & (nv < np.float32(1.5))
        bi = np.minimum((nv[sel] * np.float32(_lib.COHORT_BINS / 1.5)).astype(np.int64), 1023)
        exp_h += np.bincount(bi, minlength=_lib.COHORT_BINS).astype(np.uint64)
    assert np.array_equal(h, exp_h)


def test_cohort_rows_around_the_sample_size():
    """k_cohort_search's rows for masked counts below, at and above its 4096-key LDS sample (one
    sample per key below it) and a count large enough that each bin edge's search spans several
    keys, in one batch; summed by k_cohort_sum against numpy's histogram of p99-normalised values."""
    sizes = [1, 100, 4095, 4096, 4097, 50000]
    R, C, Z = 64, 64, 16
    rng = np.random.default_rng(31)
    hp = (rng.gamma(3.0, 40.0, size=(len(sizes), R, C, Z)) + 0.5).astype(np.float32)
    mk = np.zeros((len(sizes), R * C * Z), np.uint8)
    for b, n in enumerate(sizes):
        mk[b, rng.choice(R * C * Z, n, replace=False)] = 1
    mk = mk.reshape(len(sizes), R, C, Z)
    B = _lib.Batch(R, C, Z, len(sizes))
    B.upload(hp, mk)
    B.run(B.options(do_n4=False, vox=(1.5, 1.5, 10.0), do_cohort=True))
    res = B.download()[4]
    h = B.cohort_hist()
    B.close()
    exp_h = np.zeros(_lib.COHORT_BINS, np.uint64)
    for b in range(len(sizes)):
        s = np.sort(hp[b][mk[b] > 0])
        assert np.float32(res[b].p99) == s[int(len(s) * 0.99)]
        nv = (hp[b] / np.float32(res[b].p99)).astype(np.float32)[mk[b] > 0]
        sel = (nv >= 0) & (nv < np.float32(1.5))
        bi = np.minimum((nv[sel] * np.float32(_lib.COHORT_BINS / 1.5)).astype(np.int64), 1023)
        exp_h += np.bincount(bi, minlength=_lib.COHORT_BINS).astype(np.uint64)
    assert np.array_equal(h, exp_h)


# ---- rendering after the hot path (oracle parity unpinned) -----------
def _render_case(R, C, Z, seed):
    rng = np.random.default_rng(seed)
    i, j, k = np.meshgrid(np.arange(R), np.arange(C), np.arange(Z), indexing="ij")
    mask = (((i - R / 2) / (0.35 * R)) ** 2 + ((j - C / 2) / (0.3 * C)) ** 2 <= 1) & (k >= 1) & (k < Z - 1)
    n4 = (rng.normal(10, 4, (R, C, Z)) * mask).astype(np.float32)
    n4[0, 0, 0] = -25.0
    defect = (mask & (rng.random((R, C, Z)) < 0.2)).astype(np.float64)
    hp = rng.gamma(3.0, 2.0, (R, C, Z)).astype(np.float32)
    proton = rng.normal(100, 20, (R, C, Z))
    mb = np.zeros((R, C, Z))
    mb[1:-1, 1:-1] = (mask[2:, 1:-1] != mask[:-2, 1:-1]) | (mask[1:-1, 2:] != mask[1:-1, :-2])
    ci = np.where(defect > 0, rng.uniform(0.0, 39.9, (R, C, Z)), 0.0)
    return mask.astype(np.float64), n4, defect, hp, proton, mb, ci


@pytest.mark.parametrize("shape,seed", [((40, 36, 9), 1), ((33, 50, 7), 2), ((128, 128, 24), 3)])
def test_overlay_vs_oracle(shape, seed):
    from oracle import export_oracle as E
    _, n4, defect, *_ = _render_case(*shape, seed)
    assert np.array_equal(_lib.overlay(n4, defect), E.overlay_rgb(n4, defect))
    flat = np.full_like(n4, 2.0)   # max == min: normalize returns x (uint8 wrap of 510)
    assert np.array_equal(_lib.overlay(flat, defect), E.overlay_rgb(flat, defect))
    d2 = defect.copy()
    d2[d2 > 0] = 2.0               # defect values other than 0/1: neither branch of :389
    assert np.array_equal(_lib.overlay(n4, d2), E.overlay_rgb(n4, d2))


@pytest.mark.parametrize("shape,seed", [((40, 36, 9), 1), ((33, 50, 7), 2), ((128, 128, 24), 3)])
def test_montage_vs_oracle(shape, seed):
    from oracle import export_oracle as E
    mask, n4, defect, hp, proton, mb, ci = _render_case(*shape, seed)
    pal = parula()   # the reference's own 64 x 3 table (parula.npy, read by screenShot :466)
    rr, cc, ss = E.crop_to_data(mask, border=5)
    crop = (rr[0], len(rr), cc[0], len(cc), ss[0], len(ss))
    for c in (ci, None):
        got = _lib.montage(proton, hp, n4, mb, defect, c, pal, crop)
        assert np.array_equal(got, E.screenshot_image(proton, hp, n4, mask, mb, defect, c, pal))
    with pytest.raises(IndexError):   # int(CI * 64 / 40) past the 64-row table
        _lib.montage(proton, hp, n4, mb, defect, ci * 2, pal, crop)


def test_export_class_methods(tmp_path):
    from oracle import export_oracle as E
    from vent_analysis_amd import Vent_Analysis
    from vent_analysis_amd import dicom
    mask, n4, defect, hp, proton, mb, ci = _render_case(48, 40, 8, 4)
    v = Vent_Analysis(xenon_array=hp, mask_array=mask, proton_array=proton, vox=(1.5, 1.5, 10.0))
    v.calculate_VDP()
    rgb = v.exportDICOM(None)
    assert np.array_equal(rgb, E.overlay_rgb(v.N4HPvent, v.defectArray))
    ds = dicom.Dataset()
    v.exportDICOM(ds, save_dir=str(tmp_path), forPACS=False)
    back = dicom.dcmread(tmp_path / f"{v.metadata['PatientName']}_defectDICOM.dcm")
    assert back.Rows == 48 and back.NumberOfFrames == 8 and back["PixelData"].value == rgb.tobytes()
    pal = parula()   # the reference's own 64 x 3 table (parula.npy, read by screenShot :466)
    img = v.screenShot(path=str(tmp_path / "shot.png"), parula=pal)
    exp = E.screenshot_image(v.proton, v.HPvent, v.N4HPvent, v.mask, v.mask_border, v.defectArray,
                             None, pal)
    assert np.array_equal(img, exp) and (tmp_path / "shot.png").exists()
    from PIL import Image   # the PNG: the montage plus the reference's white text
    png = np.asarray(Image.open(tmp_path / "shot.png").convert("RGB"))
    assert png.shape == img.shape and (png != img).any()
    diff = (png != img).any(axis=2)
    assert (png[diff] >= img[diff]).all()


# ---- grid form: one study over G cooperating workgroups (k_n4_studyg) ------------------------------
def _run_one(X, M, mode, **kw):
    return _run_batch(X[None], M.astype(np.uint8)[None], mode, **kw)


@pytest.mark.parametrize("conv_mode", [0, 1])
@pytest.mark.parametrize("shape,seed", [((256, 256, 24), 7), ((128, 128, 24), 0), ((96, 112, 20), 5),
                                        ((64, 64, 64), 6)])
def test_n4_grid_vs_oracle_and_sweeps(shape, seed, conv_mode):
    """n4_mode=3 (k_n4_studyg, the default for a batch of one study) against the C oracle, and
    against the per-iteration sweep driver bit for bit (the same S1-S9 operations): N4HPvent,
    iteration counts and convergence values identical, the VDP maps identical."""
    X, M = synth_volume(*shape, seed)
    ref, its_ref, conv_ref = native.n4(X, M, conv_mode=conv_mode)
    g = _run_one(X, M, "grid", conv_mode=conv_mode)
    assert_n4_matches(g[0][0], g[4][0].n4_iters[:4], g[4][0].n4_conv[:4], ref, its_ref, conv_ref,
                      conv_mode, (shape, seed, "grid"))
    s = _run_one(X, M, "sweep", conv_mode=conv_mode)
    assert np.array_equal(g[0], s[0]) and np.array_equal(g[1], s[1]) and np.array_equal(g[3], s[3])
    assert list(g[4][0].n4_iters[:4]) == list(s[4][0].n4_iters[:4])
    assert g[4][0].n4_conv[:4] == s[4][0].n4_conv[:4]


@pytest.mark.parametrize("G", ["1", "2", "5", "13", "40"])
def test_n4_grid_any_workgroup_count(G, monkeypatch):
    """The grid form's cross-workgroup sums (histogram counts and o-weights, 128-bit lattice
    numerators, range records, the grid PC) are order-free integers: any workgroup count gives the
    same field bit for bit, run after run (VH_STG_G)."""
    X, M = synth_volume(128, 128, 24, 3)
    monkeypatch.delenv("VH_STG_G", raising=False)
    base = _run_one(X, M, "grid")
    monkeypatch.setenv("VH_STG_G", G)
    for _ in range(2):
        o = _run_one(X, M, "grid")
        assert np.array_equal(o[0], base[0]) and np.array_equal(o[1], base[1])
        assert list(o[4][0].n4_iters[:4]) == list(base[4][0].n4_iters[:4])
        assert o[4][0].n4_conv[:4] == base[4][0].n4_conv[:4]


def test_n4_grid_empty_and_tiny_masks():
    """A study with no mask voxel (n < 2: the field stays zero, N4HPvent = HPvent) and one with a
    handful, on the grid form."""
    X, M = synth_volume(64, 64, 16, 7)
    e = _run_one(X, np.zeros_like(M), "grid")
    assert e[4][0].n_mask == 0 and np.array_equal(e[0][0], X)
    M2 = np.zeros_like(M)
    M2[30:33, 30:32, 5:7] = 1
    ref, its, conv = native.n4(X, M2)
    t = _run_one(X, M2, "grid")
    assert_n4_matches(t[0][0], t[4][0].n4_iters[:4], t[4][0].n4_conv[:4], ref, its, conv, 0, "tiny")


def test_class_pooled_batch_reuse_across_studies():
    """calculate_VDP reuses one pooled device batch per shape (_lib.pooled_batch): study after study
    through the class gives what a fresh batch gives for each, N4 field and maps bit for bit."""
    from vent_analysis_amd import Vent_Analysis
    vox = (1.5, 1.5, 10.0)
    for seed in (4, 5, 4):
        X, M = synth_volume(96, 80, 16, seed)
        v = Vent_Analysis(xenon_array=X, mask_array=M, vox=vox)
        v.calculate_VDP()
        n4, d, bo, lb, res = _run_batch(X[None], M.astype(np.uint8)[None], "auto")
        assert np.array_equal(v.N4HPvent, n4[0]) and np.array_equal(v.defectArray, d[0])
        assert list(v.n4_iterations) == list(res[0].n4_iters[:4])


def test_n4_grid_several_studies_one_launch_each():
    """n4_mode=3 on a batch of three studies (one cooperative launch per study, vol0 = v, the same
    per-launch global state reused): each study equals the oracle and the sweeps."""
    hp, mk = synth_batch(96, 112, 20, 3, base_seed=40)
    g = _run_batch(hp, mk, "grid")
    s = _run_batch(hp, mk, "sweep")
    assert np.array_equal(g[0], s[0]) and np.array_equal(g[1], s[1])
    for b in range(3):
        ref, its_ref, conv_ref = native.n4(hp[b], mk[b])
        assert_n4_matches(g[0][b], g[4][b].n4_iters[:4], g[4][b].n4_conv[:4], ref, its_ref, conv_ref, 0,
                          ("grid batch", b))


@pytest.mark.parametrize("driver", ["sweep", "grid"])
@pytest.mark.parametrize("nb", [1, 2])
def test_n4_studies_smaller_than_the_pc_block_count(driver, nb):
    """Studies of fewer voxels than PC's 1024 blocks (the block layout P of a tiny study is shorter
    than one row of blocks: empty blocks must not read past it), one with an empty mask beside it."""
    hp, mk = synth_batch(8, 10, 6, nb, base_seed=50)
    mk[:, 2:6, 3:8, 1:5] = 1
    if nb == 2:
        mk[1] = 0
    n4, d, _, _, res = _run_batch(hp, mk, driver)
    ref, its, conv = native.n4(hp[0], mk[0])
    assert_n4_matches(n4[0], res[0].n4_iters[:4], res[0].n4_conv[:4], ref, its, conv, 0, ("tiny", driver))
    if nb == 2:
        assert np.array_equal(n4[1], hp[1])
