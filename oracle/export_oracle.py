"""CPU restatement (numpy) of the rendering that follows the hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module; the product path (vent_analysis_amd/, csrc/export.hip) never
does.  PARITY UNPINNED: the reference's tests hold no fixtures for these methods, and running the
reference to generate some was denied in round 2; the restatement follows the cited
lines and is checked against hand-derived properties (tests/test_export_oracle.py).

  normalize          Vent_Analysis.py:233-237 (and the local copy in screenShot, :460-464)
  overlay_rgb        exportDICOM pixel data, Vent_Analysis.py:387-393 (forPACS=False transpose)
  crop_to_data       Vent_Analysis.cropToData, :430-456 (index-0 quirk kept: np.multiply by the
                     index list makes row / col / slice 0 never "non-empty")
  screenshot_image   screenShot's montage array before the text overlay, :467-495
"""
from __future__ import annotations

import numpy as np


def normalize(x):
    """Vent_Analysis.py:233-237: (x - min) / (max - min) in x's own dtype; x itself if flat."""
    if (np.max(x) - np.min(x)) == 0:
        return x
    return (x - np.min(x)) / (np.max(x) - np.min(x))


def overlay_rgb(n4, defect):
    """exportDICOM (Vent_Analysis.py:387-393): uint8 [Z][R][C][3], slices first as written."""
    BW = (normalize(np.abs(n4)) * (2 ** 8 - 1)).astype(np.uint8)
    rgb = np.zeros(n4.shape + (3,), dtype=np.uint8)
    rgb[..., 0] = BW * (defect == 0) + 255 * (defect == 1)
    rgb[..., 1] = BW * (defect == 0)
    rgb[..., 2] = BW * (defect == 0)
    return np.transpose(rgb, (2, 0, 1, 3))


def crop_to_data(A, border=0, border_slices=False):
    """Vent_Analysis.cropToData (:430-456): (row range, col range, slice range) as lists."""
    slices = np.multiply(np.sum(np.sum(A, axis=0), axis=0) > 0, list(range(0, A.shape[2])))
    rows = np.multiply(np.sum(np.sum(A, axis=1), axis=1) > 0, list(range(0, A.shape[0])))
    cols = np.multiply(np.sum(np.sum(A, axis=2), axis=0) > 0, list(range(0, A.shape[1])))
    slices = [x for x in range(0, A.shape[2]) if slices[x]]
    rows = [x for x in range(0, A.shape[0]) if rows[x]]
    cols = [x for x in range(0, A.shape[1]) if cols[x]]
    if border_slices:
        s0, s1 = max(slices[0] - border, 0), min(slices[-1] + border + 1, A.shape[2])
    else:
        s0, s1 = max(slices[0], 0), min(slices[-1] + 1, A.shape[2])
    r0, r1 = max(rows[0] - border, 0), min(rows[-1] + border + 1, A.shape[0])
    c0, c1 = max(cols[0] - border, 0), min(cols[-1] + border + 1, A.shape[1])
    return list(range(r0, r1)), list(range(c0, c1)), list(range(s0, s1))


def _montage(images, grid_shape):
    """skimage.util.montage(images, grid_shape, padding_width=0, fill=0) for equal 2-D images:
    image k at grid cell (k // ncols, k % ncols)."""
    nr, nc = grid_shape
    h, w = images[0].shape
    out = np.zeros((nr * h, nc * w), dtype=np.result_type(*images))
    for k, im in enumerate(images):
        r, c = divmod(k, nc)
        out[r * h:(r + 1) * h, c * w:(c + 1) * w] = im
    return out


def screenshot_image(proton, hp, n4, mask, mask_border, defect, ci, parula):
    """screenShot (:467-495): uint8(IMAGE * 255), IMAGE the 7 x ns RGB montage.  ci None = the
    reference's blank CI panel (its except branch)."""
    rr, cc, ss = crop_to_data(mask, border=5)
    ix = np.ix_(rr, cc, ss)
    blank = np.zeros_like(hp[ix])
    P = normalize(proton[ix])
    HP = normalize(hp[ix])
    N4 = normalize(n4[ix])
    border = normalize(mask_border[ix]) > 0
    defArr = defect[ix] > 0
    CI = ci[ix] if ci is not None else blank
    t = CI * 64 / 40
    if np.isnan(t).any():
        raise ValueError("cannot convert float NaN to integer")
    idx = t.astype(np.int64)                       # int(): truncation toward zero
    CIred, CIgreen, CIblue = parula[idx, 0], parula[idx, 1], parula[idx, 2]   # IndexError
    R3 = np.concatenate((blank, blank, P, HP, N4 * (~border) + 0 * border, N4 * (~defArr) + defArr,
                         N4 * (CI == 0) + CIred * (CI > 0)), axis=2)
    G3 = np.concatenate((blank, blank, P, HP, N4 * (~border) + 1 * border, N4 * (~defArr),
                         N4 * (CI == 0) + CIgreen * (CI > 0)), axis=2)
    B3 = np.concatenate((blank, blank, P, HP, N4 * (~border) + 1 * border, N4 * (~defArr),
                         N4 * (CI == 0) + CIblue * (CI > 0)), axis=2)
    ns = N4.shape[2]
    mont = [_montage([A[:, :, k] for k in range(A.shape[2])], (7, ns)) for A in (R3, G3, B3)]
    return np.uint8(np.stack(mont, axis=2) * 255)
