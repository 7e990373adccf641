"""The study kernel's bin minimum without the raster scan (n4_shared.h r3_bin_min).

ITK's histogram range loop (reference path: SimpleITK N4BiasFieldCorrectionImageFilter, the
`if (u > max) max = u; else if (u < min) min = u;` scan restated in oracle/n4_oracle.c) skips
every "record" voxel.  r3_bin_min claims that minimum equals the multiset of the three smallest
values with the initial strictly increasing raster run taken out, whenever the run ends within the
first 16 voxels and leaves something of the triple.  This checks that claim (host restatement of
the device function) against the scan itself on random arrays rich in ties and rising prefixes.
"""
import numpy as np

NFIRST = 16  # n4_study.hip ST_NFIRST


def itk_min(u):
    mx, mn = -np.float32(np.finfo(np.float32).max), np.float32(np.finfo(np.float32).max)
    for v in u:
        if v > mx:
            mx = v
        elif v < mn:
            mn = v
    return mn


def r3_bin_min(u):
    """Mirror of the device function: returns None where the kernel takes the raster scan."""
    tri = sorted(u)[:3]
    tri += [np.float32(np.finfo(np.float32).max)] * (3 - len(tri))
    first = list(u[:NFIRST])
    if len(first) < 3:
        return None
    K = 1
    while K < len(first) and first[K] > first[K - 1]:
        K += 1
    if K == len(first) or not first[K] <= first[K - 1]:
        return None
    j = 0
    for m in tri:
        while j < K and first[j] < m:
            j += 1
        if j < K and first[j] == m:
            j += 1
            continue
        return m
    return None


def test_run_removal_matches_itk_scan():
    rng = np.random.default_rng(7)
    hit = 0
    for trial in range(4000):
        n = int(rng.integers(3, 60))
        levels = int(rng.integers(2, 12))
        u = rng.integers(0, levels, n).astype(np.float32)
        if trial % 3 == 0:  # a rising prefix of random length
            r = int(rng.integers(1, min(n, 20) + 1))
            u[:r] = np.sort(rng.choice(np.arange(-20, 40), r, replace=False)).astype(np.float32)
        got = r3_bin_min(u)
        if got is not None:
            hit += 1
            assert got == itk_min(u), (u, got, itk_min(u))
    assert hit > 2000  # the fast form covers most cases


def test_old_form_cases_agree():
    # runs of 1 and 2: the r1/r2g forms (u1 out of the triple; u1 < u2 out of it)
    for u in ([3, 1, 2, 5], [1, 1, 0, 7], [1, 2, 2, 0], [1, 2, 1, 1], [0, 5, 0, 9]):
        a = np.array(u, np.float32)
        assert r3_bin_min(a) == itk_min(a)
