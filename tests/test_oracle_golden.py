"""CPU: the oracle restatement against the reference's own outputs (tests/golden, produced by
running /root/reference/Vent_Analysis.py + CI.py on the same inputs) and against numpy/scipy."""
import numpy as np
import pytest
from scipy.signal import medfilt2d

from conftest import GOLDEN, golden_files, load_case
from oracle import native, vdp_oracle as O
from vent_analysis_amd.sphere import compact_table, sphere_pix

GOLD = golden_files()


@pytest.mark.parametrize("path", GOLD, ids=lambda p: p.split("/")[-1])
def test_oracle_vdp_bit_exact_vs_reference(path):
    X, M, vox, exp, _ = load_case(path)
    r = O.calculate_vdp(X, M, vox, HP=X)          # N4 = identity, as the goldens were made
    assert np.array_equal(r["defectArray"], exp["defect"])
    assert np.array_equal(r["defectBorder"], exp["defect_border"])
    assert np.array_equal(O.calculate_border(M), exp["mask_border"])
    assert np.array_equal(r["defectArrayLB"], exp["lb"])
    for k in ("VDP", "VDP_lb", "DefectVolume", "SNR", "mean_anchor", "p99"):
        assert r[k] == exp[k], k
    assert O.volume_litres(np.sum(M == 1), vox) == exp["LungVolume"]


@pytest.mark.parametrize("path", [p for p in GOLD if "ci_values" in np.load(p)],
                         ids=lambda p: p.split("/")[-1])
def test_oracle_ci_bit_exact_vs_reference(path):
    X, M, vox, exp, _ = load_case(path)
    d = exp["defect"]
    ci, shell = native.ci(d, compact_table(sphere_pix(vox, 50), d.shape), vox)
    assert np.array_equal(ci[d > 0], exp["ci_values"])
    assert np.all(ci[d == 0] == 0) and np.all(shell[d == 0] == -1)
    assert O.ci_scalar(ci[d > 0]) == exp["CI"]


def test_mean_anchor_vectors():
    g = np.load(f"{GOLDEN}/mean_anchor.npz")
    v, off = g["values"], g["offsets"]
    for i, m in enumerate(g["means"]):
        assert O.mean_f32(v[off[i]:off[i + 1]]) == m, (i, off[i + 1] - off[i])


@pytest.mark.parametrize("seed", range(6))
def test_mean_and_std_match_numpy(seed):
    rng = np.random.default_rng(seed)
    for n in rng.integers(1, 50000, 8):
        x = (rng.standard_normal(n) * 30 + 100).astype(np.float32)
        assert O.mean_f32(x) == np.mean(x)
        assert O.std_f32(x) == np.std(x)
        assert O.sum_f32(x) == np.sum(x)


def test_medfilt_matches_scipy():
    rng = np.random.default_rng(1)
    for shape in [(5, 7, 3), (32, 17, 4), (64, 64, 2)]:
        b = (rng.random(shape) < 0.5).astype(np.float64)
        ref = np.stack([medfilt2d(b[:, :, k]) for k in range(shape[2])], axis=2)
        assert np.array_equal(O.medfilt3x3_binary(b), ref)
    one = np.ones((4, 5, 1))
    out = O.medfilt3x3_binary(one)[:, :, 0]
    assert out.sum() == 20 - 4 and out[0, 0] == out[0, -1] == out[-1, 0] == out[-1, -1] == 0


def test_border_matches_np_gradient():
    rng = np.random.default_rng(2)
    for shape in [(3, 4, 2), (20, 31, 3)]:
        a = (rng.random(shape) < 0.4).astype(np.float64)
        ref = np.zeros(shape)
        for k in range(shape[2]):
            g = np.gradient(a[:, :, k])
            ref[:, :, k] = (g[0] != 0) + (g[1] != 0)
        assert np.array_equal(O.calculate_border(a), ref)
    dot = np.zeros((5, 5, 1))
    dot[2, 2] = 1
    b = O.calculate_border(dot)[:, :, 0]
    assert b[2, 2] == 0 and b[1, 2] == b[3, 2] == b[2, 1] == b[2, 3] == 1


def test_lb_classes_edges():
    e = np.array([0.0, 0.16, np.nextafter(np.float32(0.16), 1), 0.34, 0.52, 0.7, 0.88,
                  np.nextafter(np.float32(0.88), 1), 5.0, np.nan], np.float32)
    assert list(O.lb_classes(e)) == [1, 1, 2, 2, 3, 4, 5, 6, 6, 0]


def test_snr_noise_region_quirks():
    """rr/ss substitute 0 for empty rows/slices; cc drops the last masked column."""
    m = np.zeros((50, 10, 4))
    m[22:30, 3:7, 1:3] = 1
    nm = O.noise_mask(m)
    assert not nm[:20].any() and not nm[30:].any()
    box = np.zeros_like(nm)
    rows = [0] + list(range(22, 30))
    for r in rows:
        box[r, 3:6][:, [0, 1, 2]] = True
    exp = np.ones(m.shape, bool)
    rr = np.array([0] + list(range(22, 30)))
    exp[np.ix_(rr, np.arange(3, 6), np.array([0, 1, 2]))] = False
    exp[:20] = False
    exp[30:] = False
    assert np.array_equal(nm, exp)


def test_medfilt3d_matches_scipy_ndimage():
    from scipy.ndimage import median_filter
    rng = np.random.default_rng(3)
    for shape in [(6, 7, 5), (20, 17, 9), (9, 9, 1)]:
        b = (rng.random(shape) < 0.5).astype(np.float64)
        ref = median_filter(b, size=3, mode="constant", cval=0.0)
        assert np.array_equal(O.medfilt3d_binary(b), ref)


def test_border3d_matches_np_gradient():
    rng = np.random.default_rng(4)
    for shape in [(3, 4, 2), (12, 9, 7)]:
        a = (rng.random(shape) < 0.4).astype(np.float64)
        g = np.gradient(a)
        ref = ((g[0] != 0) | (g[1] != 0) | (g[2] != 0)).astype(np.float64)
        assert np.array_equal(O.calculate_border3d(a), ref)
    one = np.zeros((5, 5, 1))
    one[2, 2, 0] = 1
    assert np.array_equal(O.calculate_border3d(one), O.calculate_border(one))


@pytest.mark.parametrize("path", GOLD, ids=lambda p: p.split("/")[-1])
def test_literal_oracle_vs_reference(path):
    """calculate_vdp_literal (scipy's medfilt2d, the reference's expressions on any mask) gives
    the reference's outputs on every golden case."""
    X, M, vox, exp, _ = load_case(path)
    r = O.calculate_vdp_literal(X, M, vox)
    assert np.array_equal(r["defectArray"], exp["defect"])
    assert np.array_equal(r["defectBorder"], exp["defect_border"])
    assert np.array_equal(r["defectArrayLB"], exp["lb"])
    for k in ("VDP", "VDP_lb", "DefectVolume", "mean_anchor", "p99"):
        assert r[k] == exp[k], k


@pytest.mark.parametrize("v", [255, 2, 1.5])
def test_literal_oracle_single_value_mask(v):
    """A 0/v mask (mask DICOM folders often hold 0/255): the maps scale by v, VDP is unchanged,
    and the reference's `== 1` / `== 2` tests change DefectVolume and VDP_lb."""
    path = [p for p in GOLD if "vdp_edge" in p][0]
    X, M, vox, exp, _ = load_case(path)
    r = O.calculate_vdp_literal(X, M * v, vox)
    assert np.array_equal(r["defectArray"], exp["defect"] * np.float64(v))
    assert np.array_equal(r["defectBorder"], exp["defect_border"])
    assert np.array_equal(r["defectArrayLB"], exp["lb"] * np.float64(v))
    assert r["VDP"] == exp["VDP"]
    assert r["DefectVolume"] == (exp["DefectVolume"] if v == 1 else 0.0)
    lb = exp["lb"] * np.float64(v)
    assert r["VDP_lb"] == 100 * np.sum((lb == 1) * 1 + (lb == 2) * 1) / np.sum(M * v)
    if v == 255:
        assert r["VDP_lb"] == 0.0
