"""CPU: the build-defined k-means VDP (the reference only imports KMeans,
Vent_Analysis.py:19, 259-261) pinned against scikit-learn's Lloyd with the same initial centres."""
import numpy as np
import pytest

from oracle import vdp_oracle as O
from vent_analysis_amd.synth import synth_volume

sklearn = pytest.importorskip("sklearn.cluster")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_kmeans_matches_sklearn_lloyd(seed):
    X, M = synth_volume(96, 96, 20, seed)
    s = np.sort(X[M > 0])
    counts, centres, it = O.kmeans_1d_sorted(s)
    n = s.size
    init = np.array([[float(s[(n * (2 * j + 1)) // 8])] for j in range(4)])
    km = sklearn.KMeans(n_clusters=4, init=init, n_init=1, algorithm="lloyd", tol=0.0,
                        max_iter=300).fit(s.astype(np.float64).reshape(-1, 1))
    sk_counts = np.bincount(km.labels_, minlength=4)
    order = np.argsort(km.cluster_centers_[:, 0])
    assert np.array_equal(sk_counts[order], counts)
    assert np.allclose(km.cluster_centers_[order, 0], centres, rtol=1e-9)


def test_kmeans_clusters_are_sorted_intervals():
    rng = np.random.default_rng(0)
    s = np.sort(np.concatenate([rng.normal(20, 3, 3000), rng.normal(80, 5, 5000),
                                rng.normal(150, 8, 5000), rng.normal(220, 9, 4000)]).astype(np.float32))
    counts, centres, _ = O.kmeans_1d_sorted(s)
    assert counts.sum() == s.size and np.all(np.diff(centres) > 0)
    assert abs(counts[0] - 3000) < 30


def _sk_low_count(s):
    """scikit-learn 1.7.2 Lloyd from the oracle's initial centres: voxels in the lowest non-empty
    cluster (relocated clusters may repeat a centre value, so the non-empty ones are compared)."""
    n = s.size
    init = np.array([[float(s[(n * (2 * j + 1)) // 8])] for j in range(4)])
    km = sklearn.KMeans(n_clusters=4, init=init, n_init=1, algorithm="lloyd", tol=0.0,
                        max_iter=300).fit(s.astype(np.float64).reshape(-1, 1))
    cnt = np.bincount(km.labels_, minlength=4)
    ne = np.flatnonzero(cnt > 0)
    return int(cnt[ne[np.argmin(km.cluster_centers_[ne, 0])]])


@pytest.mark.filterwarnings("ignore::sklearn.exceptions.ConvergenceWarning")
@pytest.mark.parametrize("nvals", [2, 3])
def test_kmeans_degenerate_inputs_match_sklearn(nvals):
    """two- and three-valued data leave clusters empty (equal initial centres).
    The oracle's rule (empty clusters take the value farthest from its centre, scikit-learn's
    relocation with the tie order fixed) gives every value a cluster of its own, as scikit-learn
    1.7.2 does: VDP_km counts the smallest value, on 150 random inputs per case (proportions from
    0.1 % to 99 %, sizes 20-3000, float32 values of several magnitudes)."""
    rng = np.random.default_rng(100 + nvals)
    for trial in range(150):
        vals = np.sort(rng.choice(np.arange(1, 30), nvals, replace=False)).astype(np.float32)
        vals = (vals * np.float32([1.0, 0.37, 1e-3, 250.0][trial % 4])).astype(np.float32)
        p = rng.dirichlet(np.ones(nvals) * rng.uniform(0.2, 3))
        n = int(rng.integers(20, 3000))
        s = np.sort(rng.choice(vals, n, p=p)).astype(np.float32)
        counts, centres, _ = O.kmeans_1d_sorted(s)
        low = O.kmeans_low_count(counts)
        assert low == int((s == s[0]).sum()), (trial, vals, p, n, counts)
        assert low == _sk_low_count(s), (trial, vals, p, n, counts)
        assert np.all(np.diff(centres) >= 0)


def test_kmeans_two_values_half_half():
    """The GPU adversarial case (tests/test_gpu_parity.py two_values): 1.5 / 2.5 at random."""
    rng = np.random.default_rng(7)
    s = np.sort(rng.choice(np.float32([1.5, 2.5]), 20000)).astype(np.float32)
    counts, centres, _ = O.kmeans_1d_sorted(s)
    assert O.kmeans_low_count(counts) == int((s == 1.5).sum()) == _sk_low_count(s)
