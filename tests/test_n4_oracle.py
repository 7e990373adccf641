"""CPU: known-answer tests for the N4 restatement.  SimpleITK is not
installable offline, so N4 parity with the reference is UNPINNED; these tests pin the oracle's
behaviour to properties any correct N4 has, and the GPU is then checked against the oracle."""
import numpy as np
import pytest

from oracle import native
from vent_analysis_amd.synth import synth_volume


def log_slope(img, mask, R, sel=None):
    i = np.broadcast_to(np.arange(R)[:, None, None], img.shape)
    sel = (mask > 0) if sel is None else sel
    return np.polyfit(i[sel], np.log(img[sel]), 1)[0] * R


def phantom(R=64, C=64, Z=16, seed=0, amp=0.5):
    """Two-class piecewise-constant tissue times a smooth multiplicative bias exp(b)."""
    rng = np.random.default_rng(seed)
    i, j, k = np.meshgrid(np.arange(R), np.arange(C), np.arange(Z), indexing="ij")
    mask = (((i - R / 2) / (0.4 * R)) ** 2 + ((j - C / 2) / (0.4 * C)) ** 2 +
            ((k - Z / 2) / (0.45 * Z)) ** 2) <= 1
    tissue = np.where((i // 8 + j // 8) % 2 == 0, 100.0, 160.0)
    b = amp * (i / R - 0.5) + 0.3 * amp * np.sin(np.pi * j / C)
    img = (tissue * np.exp(b) * (1 + 0.01 * rng.standard_normal(mask.shape))).astype(np.float32)
    img[~mask] = rng.rayleigh(5, (~mask).sum()).astype(np.float32)
    return img, mask.astype(np.uint8), b


def test_removes_smooth_bias():
    X, M = synth_volume(64, 64, 16, 0)
    out, its, conv = native.n4(X, M)
    healthy = (M > 0) & (X > 100)          # exclude the x0.2 ventilation defects
    assert abs(log_slope(X, M, 64, healthy)) > 0.3
    assert abs(log_slope(out, M, 64, healthy)) < 0.05 * abs(log_slope(X, M, 64, healthy))


def test_recovers_phantom_bias_up_to_constant():
    img, mask, b = phantom()
    out, its, _ = native.n4(img, mask)
    sel = mask > 0
    est = np.log(img[sel]) - np.log(out[sel])          # estimated log bias at masked voxels
    err = (est - est.mean()) - (b[sel] - b[sel].mean())
    assert np.std(err) < 0.25 * np.std(b[sel])


def test_iteration_counts_and_convergence():
    X, M = synth_volume(64, 64, 16, 1)
    out, its, conv = native.n4(X, M)
    assert np.all((its >= 1) & (its <= 50))
    for n, c in zip(its, conv):
        assert n == 50 or c <= 0.001


def test_max_iters_respected():
    X, M = synth_volume(48, 48, 12, 2)
    out, its, conv = native.n4(X, M, max_iters=(3, 2), conv_threshold=0.0)
    assert list(its) == [3, 2]


def test_scale_covariance():
    """N4(k I) = k N4(I): log(kI) shifts U by log k, which shifts the histogram range and the E map
    by the same amount, so residuals, lattice and bias are unchanged."""
    X, M = synth_volume(64, 64, 16, 3)
    a, ia, _ = native.n4(X, M)
    b, ib, _ = native.n4(X * np.float32(4.0), M)
    assert list(ia) == list(ib)
    assert np.max(np.abs(b / 4.0 - a) / a) < 1e-4


def test_output_outside_mask_is_bias_corrected_too():
    X, M = synth_volume(48, 48, 12, 4)
    out, _, _ = native.n4(X, M)
    ratio = X / out                                   # = exp(B) everywhere
    assert np.all(np.isfinite(ratio)) and np.all(ratio > 0)
    assert not np.allclose(ratio[M == 0], 1.0)


def test_deterministic():
    X, M = synth_volume(48, 48, 12, 5)
    a = native.n4(X, M)[0]
    b = native.n4(X, M)[0]
    assert np.array_equal(a, b)


def test_markstein_division_lemma():
    """The GPU's exact sig step (n4_shared.h pc_div) takes ITK's RN(sqr(p - mu) (N - 1) / N) as
    Markstein's correction from RN(1/N); it must equal the IEEE double division (N in [2, 2^24],
    including powers of two and their neighbours)."""
    import ctypes as ct
    f = native.lib().markstein_check
    f.restype = ct.c_int64
    assert f(ct.c_int64(4_000_000), ct.c_uint64(12345)) == 0


def itk_convergence_py(d):
    """ITK's CalculateConvergenceMeasurement with RealType = float, restated step by step in numpy
    scalars (itkN4BiasFieldCorrectionImageFilter: N += 1.0; if (N > 1.0) sigma = sigma +
    sqr(pixel - mu) * (N - 1.0) / N; mu = mu * (1.0 - 1.0 / N) + pixel / N; each right-hand side
    in double, assigned to float)."""
    f32, f64 = np.float32, np.float64
    mu = sig = N = f32(0.0)
    for x in d:
        p = f32(np.exp(f64(x)))
        N = f32(f64(N) + 1.0)
        if f64(N) > 1.0:
            q = f32(p - mu)
            sig = f32(f64(sig) + (f64(f32(q * q)) * (f64(N) - 1.0)) / f64(N))
        mu = f32(f64(mu) * (1.0 - 1.0 / f64(N)) + f64(f32(p / N)))
    s = f32(np.sqrt(f64(sig) / (f64(N) - 1.0)))
    return f32(s / mu)


def test_conv_welford_follows_itk_roundings():
    """S7 of the build spec (oracle conv_welford, which the GPU matches bit for bit) equals ITK's
    float recurrence with its separate double roundings, on field differences of the N4 scale."""
    import ctypes as ct
    f = native.lib().n4o_conv_welford
    f.restype = ct.c_float
    rng = np.random.default_rng(3)
    for n, scale in ((2, 1e-2), (37, 3e-3), (5000, 2e-3), (20000, 1e-3)):
        d = (rng.standard_normal(n) * scale).astype(np.float32)
        got = f(d.ctypes.data_as(ct.POINTER(ct.c_float)), ct.c_int64(n))
        assert np.float32(got) == itk_convergence_py(d), n
    # the float counter stops at 2^24 (2^24 + 1 rounds to even), which conv_welford shares
    assert np.float32(np.float64(np.float32(2.0 ** 24)) + 1.0) == np.float32(2.0 ** 24)


def _conv(mu, sig, n):
    """ITK's measure from the float state (n4_shared.h itk_conv): float sqrt of sig / (N - 1) over mu."""
    sd = np.float32(np.sqrt(np.float64(sig) / (min(float(n), 2.0 ** 24) - 1.0)))
    return np.float32(sd / np.float32(mu))


@pytest.mark.parametrize("shape,seed,nb,vary", [((64, 64, 16), 0, 1024, False),
                                                ((128, 128, 24), 17, 1024, True),
                                                ((40, 36, 9), 5, 64, False)])
def test_pc_early_decision_bound(tmp_path, monkeypatch, shape, seed, nb, vary):
    """PC's early certified decision (n4_shared.h pcw_run, PC_PRE), restated by
    oracle/n4_oracle.c n4o_pc_pre_bound: on every iteration's d sequence of an oracle N4 run the
    float mean stays within D_k of the exact running mean (the drift bound the decision rests on),
    the bound lo never exceeds ITK's float sig, muhi is at or above its float mean, so the measure
    at (RD(lo), muhi) never exceeds the true one; and it decides some iterations at the default
    threshold (those well above it)."""
    import ctypes as ct
    dump = tmp_path / "d.bin"
    monkeypatch.setenv("N4_DUMP_D", str(dump))
    X, M = synth_volume(*shape, seed, vary=vary)
    native.n4(X, M)
    raw = dump.read_bytes()
    L = native.lib()
    L.n4o_pc_pre_bound.restype = None
    off = its = decided = 0
    while off < len(raw):
        n = int(np.frombuffer(raw, np.int64, 1, off)[0])
        d = np.frombuffer(raw, np.float32, n, off + 8).copy()
        off += 8 + 4 * n
        lo, muhi, ok, dmax = ct.c_double(), ct.c_float(), ct.c_int(), ct.c_double()
        sig, mu = ct.c_float(), ct.c_float()
        L.n4o_pc_pre_bound(d.ctypes.data_as(ct.POINTER(ct.c_float)), ct.c_int64(n), ct.c_int(nb),
                           ct.byref(lo), ct.byref(muhi), ct.byref(ok), ct.byref(dmax), ct.byref(sig),
                           ct.byref(mu))
        assert ok.value == 1
        assert dmax.value <= 1.0, (its, dmax.value)          # |mu_k - m_k| <= D_k at every step
        assert lo.value <= sig.value, (its, lo.value, sig.value)
        assert muhi.value >= mu.value
        sl = np.float32(lo.value)
        if np.float64(sl) > lo.value:
            sl = np.nextafter(sl, np.float32(0))
        if lo.value > 0.0:
            assert _conv(muhi.value, sl, n) <= _conv(mu.value, sig.value, n)
            decided += _conv(muhi.value, sl, n) > np.float32(0.001)
        its += 1
    assert its >= 4 and decided >= 1


@pytest.mark.parametrize("shape,seed,nb", [((64, 64, 16), 0, 1024), ((96, 80, 12), 3, 1024),
                                           ((40, 36, 9), 5, 64)])
def test_pc_sig_lower_bound(tmp_path, monkeypatch, shape, seed, nb):
    """PC's certified decision (n4_shared.h pcw_run): the bound from stage 0's block sums never
    exceeds the float sig of ITK's recurrence, on every iteration's d sequence of an oracle N4 run,
    so a measure above the threshold at the bound (and mu one float up) proves the true one is."""
    import ctypes as ct
    dump = tmp_path / "d.bin"
    monkeypatch.setenv("N4_DUMP_D", str(dump))
    X, M = synth_volume(*shape, seed)
    native.n4(X, M)
    raw = dump.read_bytes()
    L = native.lib()
    L.n4o_pc_sig_bound.restype = None
    off = its = 0
    while off < len(raw):
        n = int(np.frombuffer(raw, np.int64, 1, off)[0])
        d = np.frombuffer(raw, np.float32, n, off + 8).copy()
        off += 8 + 4 * n
        lo, sig, mu = ct.c_double(), ct.c_float(), ct.c_float()
        L.n4o_pc_sig_bound(d.ctypes.data_as(ct.POINTER(ct.c_float)), ct.c_int64(n), ct.c_int(nb),
                           ct.byref(lo), ct.byref(sig), ct.byref(mu))
        assert 0.0 < lo.value <= sig.value, (its, lo.value, sig.value)
        sl = np.float32(lo.value)
        if np.float64(sl) > lo.value:
            sl = np.nextafter(sl, np.float32(0))
        muh = np.nextafter(np.float32(mu.value), np.float32(np.inf))
        assert _conv(muh, sl, n) <= _conv(mu.value, sig.value, n)
        assert lo.value > 0.95 * sig.value          # tight enough to decide most iterations
        its += 1
    assert its >= 4


def test_pc_sig_lower_bound_past_2_24_steps():
    """The certified decision's accumulation factor (1 - 2^-24)^(n + L + 8) (round 6, pc_accum_factor)
    stays a lower bound past 2^24 steps, where the float counter N freezes and the float sum of the
    sig increments swamps: on a config-5-sized sequence (2^25 + 12345 steps, d ~ N(0, 0.02), the grid
    PC's 262144 blocks) the bound is positive and below ITK's float sig (the linear factor it
    replaces, 1 - (n + L + 8) 2^-24, is negative there: no decision was possible)."""
    import ctypes as ct
    n = (1 << 25) + 12345
    rng = np.random.default_rng(5)
    d = (rng.standard_normal(n) * 0.02).astype(np.float32)
    L = native.lib()
    L.n4o_pc_sig_bound.restype = None
    lo, sig, mu = ct.c_double(), ct.c_float(), ct.c_float()
    nb = 262144
    L.n4o_pc_sig_bound(d.ctypes.data_as(ct.POINTER(ct.c_float)), ct.c_int64(n), ct.c_int(nb),
                       ct.byref(lo), ct.byref(sig), ct.byref(mu))
    assert 1.0 - (n + n // nb + 8.0) * 2.0 ** -24 < 0.0      # the old factor: no bound at all
    assert 0.0 < lo.value <= sig.value, (lo.value, sig.value)
    f = np.exp((n + n // nb + 8.0) * np.log1p(-2.0 ** -24))
    assert 0.1 < f < 0.2                                       # (1 - 2^-24)^n ~ e^-2


@pytest.mark.parametrize("m", [1.0, 1e3, 1e6, 2.0 ** 23, 2.0 ** 24, 3e7])
def test_pc_accum_factor_dominates_linear(m):
    """(1 - u)^m >= 1 - m u (Bernoulli): the decisions only get stronger, and the factor is positive."""
    u = 2.0 ** -24
    f = np.exp(m * np.log1p(-u)) * (1.0 - 2.0 ** -40)
    assert f > 0.0 and f >= 1.0 - m * u - 2.0 ** -39
