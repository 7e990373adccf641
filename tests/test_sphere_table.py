"""CPU: the sphere-growing table generator (CI.py:33-63) is bit-identical to the reference's cached
tables, and the CI module helpers keep the reference's index semantics."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from vent_analysis_amd import CI
from vent_analysis_amd.sphere import compact_table, radii_indices, sphere_pix

PINS = json.load(open(os.path.join(GOLDEN, "sphere_tables.json")))
TABLES = [k for k in PINS if not k.startswith("_")]


@pytest.mark.parametrize("name", TABLES)
def test_table_matches_reference_checksum(name):
    p = PINS[name]
    t = sphere_pix(p["vox"], p["radius"])
    assert t.shape == (p["rows"], 4) and t.dtype == np.float64
    assert hashlib.sha256(np.ascontiguousarray(t).tobytes()).hexdigest() == p["sha256"]
    assert len(radii_indices(t)) == p["bounds"]
    ref = os.path.join("/root/reference", name)
    if os.path.exists(ref):   # authoring container only; the GPU box has no reference
        assert np.array_equal(np.load(ref, allow_pickle=False), t)


def test_radii_indices_matches_reference_formula():
    t = sphere_pix((1.5, 1.5, 10.0), 50)
    diffs = np.diff(t[:, 0]) > 0                      # CI.py:82-85 verbatim semantics
    sr = np.where(diffs)[0] + 2
    sr = sr[sr > 0] - 1
    assert np.array_equal(CI.getRadiiIndices(t), sr)


def test_compact_table_and_duplicates():
    t = sphere_pix((1.5, 1.5, 10.0), 50)
    big = compact_table(t, (128, 128, 24))
    # s0, s1 > 100: only literal repeats (a point that float rounding puts in two shells) alias
    rows_unique = np.unique(t[:, 1:], axis=0).shape[0]
    assert big.dup.sum() == t.shape[0] - rows_unique == 4
    assert np.all(np.diff(big.bounds) > 0)
    assert np.array_equal(big.radii, t[big.bounds - 1, 0])
    small = compact_table(t, (40, 36, 9))
    lin = t[:, 1] + t[:, 2] * 40 + t[:, 3] * 40 * 36
    assert small.dup.sum() == lin.size - np.unique(lin).size


def test_px2vec_vec2px_roundtrip():
    shape = (7, 5, 3)
    for i, j, k in [(1, 1, 1), (7, 5, 3), (3, 2, 2)]:     # 1-based MATLAB-style, as vec2px
        n = CI.px2vec(i, j, k, shape)
        assert CI.vec2px(n, shape) == (i, j, k)
    assert CI.px2vec(0, 0, 0, shape) == -(7 + 35)


def test_multi_which_c_order():
    a = np.zeros((3, 4, 2))
    a[2, 1, 0] = a[0, 3, 1] = 1
    assert CI.multi_which(a).tolist() == [[0, 3, 1], [2, 1, 0]]
