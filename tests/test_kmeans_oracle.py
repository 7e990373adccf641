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
