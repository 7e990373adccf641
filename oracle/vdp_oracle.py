"""ORACLE -- test infrastructure only.  CPU restatement of the post-N4 Vent_Analysis path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / the timed CPU baseline.  The product path (vent_analysis_amd) never calls it.

Pinned against the reference itself: tests/golden/*.npz were produced by running
/root/reference/Vent_Analysis.py + CI.py on the same seeded inputs (tests/golden/make_goldens.py),
and tests/test_oracle_golden.py checks every function here bit-for-bit against them.

Each function cites the reference lines it restates.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
NUMPY_BUFSIZE = 8192   # numpy ufunc-reduction buffer: float32 add.reduce runs per 8192 elements


# ------------------------------------------------------------------------------------------------
# numpy float32 reductions (Appendix B.2) -- exact order of operations of np.add.reduce
# ------------------------------------------------------------------------------------------------
def pairwise_sum_f32(a: np.ndarray) -> F32:
    """numpy's pairwise_sum for float32 (n<8: serial; n<=128: 8 lanes + tree + tail; else split
    at n2 = n/2 - (n/2)%8).  Used by np.mean / np.sum on float32 (Vent_Analysis.py:246, 356)."""
    n = a.shape[0]
    if n < 8:
        res = F32(0.0)
        for x in a:
            res = F32(res + x)
        return res
    if n <= 128:
        r = a[:8].astype(F32, copy=True)
        i = 8
        lim = n - (n % 8)
        while i < lim:
            r = (r + a[i:i + 8]).astype(F32)
            i += 8
        res = F32(F32(F32(r[0] + r[1]) + F32(r[2] + r[3])) + F32(F32(r[4] + r[5]) + F32(r[6] + r[7])))
        while i < n:
            res = F32(res + a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return F32(pairwise_sum_f32(a[:n2]) + pairwise_sum_f32(a[n2:]))


def sum_f32(a: np.ndarray) -> F32:
    """np.add.reduce over a contiguous float32 vector: serial sum of per-8192-chunk pairwise sums,
    starting from 0."""
    a = np.ascontiguousarray(a, dtype=F32)
    s = F32(0.0)
    for o in range(0, a.shape[0], NUMPY_BUFSIZE):
        s = F32(s + pairwise_sum_f32(a[o:o + NUMPY_BUFSIZE]))
    return s


def mean_f32(a: np.ndarray) -> F32:
    """np.mean of a float32 vector: float32(float64(sum) / n)."""
    return F32(np.float64(sum_f32(a)) / np.float64(a.shape[0]))


def std_f32(a: np.ndarray) -> F32:
    """np.std (ddof 0) of a float32 vector: sqrt(mean((x - mean)^2)) in float32, numpy _var order."""
    a = np.ascontiguousarray(a, dtype=F32)
    m = mean_f32(a)
    d = (a - m).astype(F32)
    d = (d * d).astype(F32)
    v = F32(np.float64(sum_f32(d)) / np.float64(a.shape[0]))
    return F32(np.sqrt(v))


# ------------------------------------------------------------------------------------------------
# stencils (Appendix B.4, B.5)
# ------------------------------------------------------------------------------------------------
def calculate_border(A: np.ndarray) -> np.ndarray:
    """Vent_Analysis.calculateBorder (Vent_Analysis.py:225-231): per slice, np.gradient != 0 along
    rows OR cols.  Interior: f[i+1] != f[i-1]; edges: one-sided difference.  Returns float64 0/1."""
    A = np.asarray(A, dtype=np.float64)
    R, C = A.shape[0], A.shape[1]
    gr = np.zeros(A.shape, bool)
    gc = np.zeros(A.shape, bool)
    gr[1:R - 1] = A[2:] != A[:R - 2]
    gr[0] = A[1] != A[0]
    gr[R - 1] = A[R - 1] != A[R - 2]
    gc[:, 1:C - 1] = A[:, 2:] != A[:, :C - 2]
    gc[:, 0] = A[:, 1] != A[:, 0]
    gc[:, C - 1] = A[:, C - 1] != A[:, C - 2]
    return (gr | gc).astype(np.float64)


def medfilt3x3_binary(B: np.ndarray) -> np.ndarray:
    """scipy.signal.medfilt2d(kernel 3) on each slice of a 0/1 volume (Vent_Analysis.py:248-249):
    zero padding, so the median of 9 binary values is 1 iff at least 5 are 1."""
    b = (np.asarray(B) != 0).astype(np.int32)
    p = np.pad(b, ((1, 1), (1, 1), (0, 0)))
    cnt = np.zeros(b.shape, np.int32)
    R, C = b.shape[0], b.shape[1]
    for dr in range(3):
        for dc in range(3):
            cnt += p[dr:dr + R, dc:dc + C]
    return (cnt >= 5).astype(np.float64)


def medfilt3d_binary(B: np.ndarray) -> np.ndarray:
    """Build-defined 3-D morphology (BASELINE config 5): 3x3x3 median of a 0/1 volume with zero
    padding = 1 iff at least 14 of the 27 neighbours are 1 (scipy.ndimage.median_filter(size=3,
    mode='constant'))."""
    b = (np.asarray(B) != 0).astype(np.int32)
    p = np.pad(b, 1)
    cnt = np.zeros(b.shape, np.int32)
    R, C, Z = b.shape
    for dr in range(3):
        for dc in range(3):
            for dz in range(3):
                cnt += p[dr:dr + R, dc:dc + C, dz:dz + Z]
    return (cnt >= 14).astype(np.float64)


def calculate_border3d(A: np.ndarray) -> np.ndarray:
    """Build-defined 3-D border: np.gradient != 0 along rows, cols OR slices (one-sided at the
    edges, as calculate_border); an axis of length 1 contributes nothing.  Returns float64 0/1."""
    A = np.asarray(A, dtype=np.float64)
    out = calculate_border(A) != 0
    Z = A.shape[2]
    if Z > 1:
        gz = np.zeros(A.shape, bool)
        gz[:, :, 1:Z - 1] = A[:, :, 2:] != A[:, :, :Z - 2]
        gz[:, :, 0] = A[:, :, 1] != A[:, :, 0]
        gz[:, :, Z - 1] = A[:, :, Z - 1] != A[:, :, Z - 2]
        out |= gz
    return out.astype(np.float64)


# ------------------------------------------------------------------------------------------------
# SNR (Vent_Analysis.py:337-357)
# ------------------------------------------------------------------------------------------------
def noise_mask(mask: np.ndarray, FOVbuffer: int = 20) -> np.ndarray:
    """The noise region of calculate_SNR: outside the ix_(rr, cc, ss) box and the first/last
    FOVbuffer rows.  rr/ss substitute index 0 for empty rows/slices (so row/slice 0 join the box
    whenever any row/slice is empty); cc = arange(min(cc[cc>0]), max(cc)) drops the last masked
    column (Vent_Analysis.py:343-351)."""
    R, C, Z = mask.shape
    rows = mask.sum(axis=(1, 2)) > 0
    cols = mask.sum(axis=(0, 2)) > 0
    sls = mask.sum(axis=(0, 1)) > 0
    rr = np.where(rows, np.arange(R), 0)
    cc = np.where(cols, np.arange(C), 0)
    cc = np.arange(np.min(cc[cc > 0]), np.max(cc))
    ss = np.where(sls, np.arange(Z), 0)
    rin = np.zeros(R, bool)
    rin[rr] = True
    cin = np.zeros(C, bool)
    cin[cc] = True
    sin = np.zeros(Z, bool)
    sin[ss] = True
    nm = ~(rin[:, None, None] & cin[None, :, None] & sin[None, None, :])
    nm[:FOVbuffer] = False
    nm[R - FOVbuffer:] = False
    return nm


def calculate_snr(A: np.ndarray, mask: np.ndarray):
    """(mean(signal) - mean(noise)) / std(noise), in A's float dtype (float32 for float32 A)."""
    signal = A[mask > 0]
    noise = A[noise_mask(mask)]
    if A.dtype == np.float32:
        return F32(F32(mean_f32(signal) - mean_f32(noise)) / std_f32(noise))
    return (np.mean(signal) - np.mean(noise)) / np.std(noise)


# ------------------------------------------------------------------------------------------------
# VDP (Vent_Analysis.py:239-263)
# ------------------------------------------------------------------------------------------------
LB_EDGES = tuple(F32(x) for x in (0.16, 0.34, 0.52, 0.7, 0.88))


def lb_classes(nv: np.ndarray) -> np.ndarray:
    """Linear-binning class 1..6 (Vent_Analysis.py:256): x<=e0 ->1, (e0,e1] ->2, ... >e4 ->6 with
    float32 edges; NaN -> 0."""
    e = LB_EDGES
    out = np.zeros(nv.shape, np.uint8)
    out[nv <= e[0]] = 1
    for c in range(1, 5):
        out[(nv > e[c - 1]) & (nv <= e[c])] = c + 1
    out[nv > e[4]] = 6
    return out


def volume_litres(count, vox) -> float:
    """count * prod(vox/10) / 1000 (Vent_Analysis.py:166, 252)."""
    return count * np.prod(np.divide(vox, 10)) / 1000


def _km_boundary(x, clo, chi):
    """First index of sorted x whose value is strictly closer to chi than to clo (clo < chi): the
    predicate is monotone over sorted x; numpy's searchsorted bisection order."""
    lo, hi = 0, x.shape[0]
    while lo < hi:
        mid = lo + ((hi - lo) >> 1)
        if not (abs(x[mid] - chi) < abs(x[mid] - clo)):
            lo = mid + 1
        else:
            hi = mid
    return lo


def kmeans_1d_sorted(s: np.ndarray, k: int = 4, max_iter: int = 300):
    """Build-defined k-means VDP (the reference only imports KMeans,
    Vent_Analysis.py:19, and leaves the k-means VDP commented out, :259-261).  Lloyd on sorted 1-D
    float32 data (float64 arithmetic), k = 4, centres kept sorted:

    * start: the order statistics c_j = s[floor(n (2j + 1) / 2k)];
    * assign: a value joins its nearest centre; equal centres -> the lowest index (a duplicate
      centre gets no points), a value exactly between two centres -> the lower one.  Over sorted
      centres the clusters are intervals: cut_{j+1} = the first value strictly closer to the next
      larger centre value than to c_j (n when c_j is the largest);
    * stop when the cuts repeat;
    * update: c_j = the mean of cluster j.  A cluster left empty takes the value farthest from its
      own cluster's centre among clusters of >= 2 values (a cluster's farthest values are its two
      ends; ties -> the lowest index; a value at distance 0 is never taken), which leaves its
      donor's sum -- scikit-learn's empty-cluster relocation (_relocate_empty_clusters_dense) with
      its tie order fixed; an empty cluster with nothing to take keeps its centre.  Then the
      centres are sorted.

    On data with two or three distinct values every value ends in a cluster of its own, as in
    scikit-learn 1.7.2's Lloyd from the same centres (tests/test_kmeans_oracle.py pins this);
    with four or more distinct values and empty clusters, which Lloyd local minimum is reached
    depends on the relocation tie order (scikit-learn's comes from np.argpartition), so there the
    result is build-defined.  On non-degenerate data (distinct increasing centres, no empty
    cluster) the steps reduce to plain Lloyd.

    Returns (counts[k], centres[k] sorted, iterations).  VDP_km counts the lowest non-empty
    cluster (:func:`kmeans_low_count`)."""
    n = s.shape[0]
    x = s.astype(np.float64)
    c = np.array([x[(n * (2 * j + 1)) // (2 * k)] for j in range(k)])
    cum = np.concatenate([[0.0], np.cumsum(x)])
    cuts = None
    it = 0
    for it in range(1, max_iter + 1):
        newcuts = np.empty(k + 1, np.int64)
        newcuts[0], newcuts[k] = 0, n
        for j in range(k - 1):
            up = c[j + 1:][c[j + 1:] > c[j]]
            newcuts[j + 1] = _km_boundary(x, c[j], up[0]) if up.size else n
        newcuts[1:k] = np.maximum.accumulate(newcuts[1:k])
        if cuts is not None and np.array_equal(newcuts, cuts):
            break
        cuts = newcuts
        old = c.copy()
        cnt = np.diff(cuts).astype(np.int64)
        sums = np.array([cum[cuts[j + 1]] - cum[cuts[j]] for j in range(k)])
        win = [[int(cuts[j]), int(cuts[j + 1])] for j in range(k)]
        newc = c.copy()
        for j in range(k):
            if np.diff(cuts)[j] > 0:
                continue
            best, bi, bq = 0.0, -1, -1
            for q in range(k):
                a, e = win[q]
                if e - a < 2:
                    continue
                for i in (a, e - 1):
                    dd = abs(x[i] - old[q])
                    if dd > best or (dd == best and dd > 0.0 and i < bi):
                        best, bi, bq = dd, i, q
            if bi >= 0:
                newc[j] = x[bi]
                sums[bq] -= x[bi]
                cnt[bq] -= 1
                if bi == win[bq][0]:
                    win[bq][0] += 1
                else:
                    win[bq][1] -= 1
        for j in range(k):
            if cuts[j + 1] > cuts[j]:
                newc[j] = sums[j] / cnt[j]
        c = np.sort(newc)
    counts = np.diff(cuts)
    return counts, c, it


def kmeans_low_count(counts) -> int:
    """Voxels in the lowest non-empty k-means cluster (VDP_km's numerator)."""
    nz = np.flatnonzero(np.asarray(counts) > 0)
    return int(counts[nz[0]]) if nz.size else 0


def calculate_vdp(N4: np.ndarray, mask: np.ndarray, vox, thresh: float = 0.6, HP=None,
                  morph3d: bool = False):
    """Vent_Analysis.calculate_VDP after N4 (Vent_Analysis.py:245-257) + build-defined k-means.
    morph3d: build-defined 3-D median / border instead of the per-slice ones (config 5).

    Returns a dict with defectArray (f64 0/1), defectBorder (bool), defectArrayLB (f64 0..6),
    VDP, DefectVolume, VDP_lb, VDP_km, SNR (if HP given), mean_anchor, p99."""
    N4 = np.asarray(N4, dtype=F32)
    sig = np.sort(N4[mask > 0], kind="stable")                          # :245
    m = mean_f32(sig)                                                   # :246
    mn = (N4 / m).astype(F32)
    raw = (mn < F32(thresh)) * (mask != 0)                              # :249 (binary mask)
    if morph3d:
        defect = medfilt3d_binary(raw)
        border = calculate_border3d(defect) == 1
    else:
        defect = medfilt3x3_binary(raw)                                 # :248-249
        border = calculate_border(defect) == 1                          # :250
    msum = np.sum(mask)
    out = dict(defectArray=defect, defectBorder=border, mean_anchor=m)
    out["VDP"] = 100 * np.sum(defect) / msum                            # :251
    out["DefectVolume"] = volume_litres(np.sum(defect == 1), vox)       # :252
    p99 = sig[int(len(sig) * .99)]                                      # :255
    nv = (N4 / p99).astype(F32)
    lb = lb_classes(nv).astype(np.float64) * mask                       # :256
    out["defectArrayLB"] = lb
    out["p99"] = p99
    out["VDP_lb"] = 100 * np.sum((lb == 1) * 1 + (lb == 2) * 1) / msum  # :257
    counts, centres, _ = kmeans_1d_sorted(sig)
    out["VDP_km"] = 100 * kmeans_low_count(counts) / msum
    out["km_centres"] = centres
    if HP is not None:
        out["SNR"] = calculate_snr(HP, mask)
    return out


def calculate_vdp_literal(N4: np.ndarray, mask: np.ndarray, vox, thresh: float = 0.6):
    """Vent_Analysis.calculate_VDP after N4 (Vent_Analysis.py:245-257) line by line, for ANY
    numeric mask (e.g. 0/255 mask DICOMs): the signal is ``mask > 0`` (:245), the per-slice
    threshold map is multiplied by the mask itself and filtered by scipy's own ``medfilt2d``
    (the reference's third-party call, :248-249), the LB classes are multiplied by the mask
    (:256) and every scalar is the reference's expression on those arrays.  Slow (scipy per
    slice); for small cases.  Equal to calculate_vdp for 0/1 masks
    (tests/test_oracle_golden.py)."""
    from scipy.signal import medfilt2d
    N4 = np.asarray(N4, dtype=F32)
    mask = np.asarray(mask)
    sig = np.sort(N4[mask > 0], kind="stable")                          # :245 sorted(...)
    m = mean_f32(sig)                                                   # :246 np.mean
    mn = np.divide(N4, m)
    defect = np.zeros(mn.shape)
    for k in range(mask.shape[2]):                                      # :247-249
        defect[:, :, k] = medfilt2d((mn[:, :, k] < F32(thresh)) * mask[:, :, k])
    border = calculate_border(defect) == 1                              # :250
    msum = np.sum(mask)
    out = dict(defectArray=defect, defectBorder=border, mean_anchor=m)
    out["VDP"] = 100 * np.sum(defect) / msum                            # :251
    out["DefectVolume"] = volume_litres(np.sum(defect == 1), vox)       # :252
    p99 = sig[int(len(sig) * .99)]                                      # :255
    nv = np.divide(N4, p99)
    lb = lb_classes(nv).astype(np.int64) * mask                         # :256 (int * mask)
    out["defectArrayLB"] = lb
    out["p99"] = p99
    out["VDP_lb"] = 100 * np.sum((lb == 1) * 1 + (lb == 2) * 1) / msum  # :257
    return out


def ci_scalar(ci_values: np.ndarray) -> float:
    """Vent_Analysis.calculate_CI tail (Vent_Analysis.py:268-270): 95th-pct order statistic."""
    s = np.sort(ci_values)
    return s[int(0.95 * len(s))]
