"""Single-file NIfTI-1 (.nii) writer/reader for the 4-D export.

The reference exports ``build4DdataArray()`` (float32 (R, C, Z, 6): proton, HPvent, mask,
N4HPvent, defectArray, CIarray) with ``nib.save(nib.Nifti1Image(dataArray, affine=np.eye(4)),
path)`` (Vent_Analysis.py:273-290).  nibabel is not installed in this image, so this module writes
the NIfTI-1 format directly: the 348-byte header, a 4-byte empty extension flag, then the voxels
in Fortran (column-major) order from byte 352, as nibabel writes them.  Header choices follow a
fresh ``Nifti1Image`` with an affine: sform_code 2 (aligned) with srow = the affine rows,
qform_code 0 with the quaternion of the affine, pixdim from the affine's column norms, and
scl_slope / scl_inter NaN (no scaling).

Parity unpinned (nibabel absent): checked by round trips and field-by-field header checks in
tests/test_nifti.py.
"""
from __future__ import annotations

import os
import struct

import numpy as np

__all__ = ["save", "load"]

_DTYPES = {np.dtype(np.uint8): (2, 8), np.dtype(np.int16): (4, 16), np.dtype(np.int32): (8, 32),
           np.dtype(np.float32): (16, 32), np.dtype(np.float64): (64, 64),
           np.dtype(np.int8): (256, 8), np.dtype(np.uint16): (512, 16),
           np.dtype(np.uint32): (768, 32), np.dtype(np.int64): (1024, 64),
           np.dtype(np.uint64): (1280, 64)}
_CODES = {code: dt for dt, (code, _) in _DTYPES.items()}

# field name, struct format -- NIfTI-1 header, 348 bytes
_FIELDS = [("sizeof_hdr", "i"), ("data_type", "10s"), ("db_name", "18s"), ("extents", "i"),
           ("session_error", "h"), ("regular", "c"), ("dim_info", "B"), ("dim", "8h"),
           ("intent_p1", "f"), ("intent_p2", "f"), ("intent_p3", "f"), ("intent_code", "h"),
           ("datatype", "h"), ("bitpix", "h"), ("slice_start", "h"), ("pixdim", "8f"),
           ("vox_offset", "f"), ("scl_slope", "f"), ("scl_inter", "f"), ("slice_end", "h"),
           ("slice_code", "B"), ("xyzt_units", "B"), ("cal_max", "f"), ("cal_min", "f"),
           ("slice_duration", "f"), ("toffset", "f"), ("glmax", "i"), ("glmin", "i"),
           ("descrip", "80s"), ("aux_file", "24s"), ("qform_code", "h"), ("sform_code", "h"),
           ("quatern_b", "f"), ("quatern_c", "f"), ("quatern_d", "f"), ("qoffset_x", "f"),
           ("qoffset_y", "f"), ("qoffset_z", "f"), ("srow_x", "4f"), ("srow_y", "4f"),
           ("srow_z", "4f"), ("intent_name", "16s"), ("magic", "4s")]
_FMT = "<" + "".join(f for _, f in _FIELDS)
assert struct.calcsize(_FMT) == 348


def _quaternion(affine):
    """(b, c, d, qfac, pixdim[1:4]) of the rotation part (NIfTI-1 qform, method 2)."""
    M = np.asarray(affine, dtype=np.float64)[:3, :3]
    zooms = np.sqrt((M * M).sum(axis=0))
    zooms[zooms == 0] = 1.0
    R = M / zooms
    qfac = 1.0
    if np.linalg.det(R) < 0:
        R[:, 2] *= -1
        qfac = -1.0
    a = 1.0 + R[0, 0] + R[1, 1] + R[2, 2]
    if a > 0.5:
        a = 0.5 * np.sqrt(a)
        b = 0.25 * (R[2, 1] - R[1, 2]) / a
        c = 0.25 * (R[0, 2] - R[2, 0]) / a
        d = 0.25 * (R[1, 0] - R[0, 1]) / a
    else:
        xd, yd, zd = 1.0 + R[0, 0] - (R[1, 1] + R[2, 2]), 1.0 + R[1, 1] - (R[0, 0] + R[2, 2]), \
            1.0 + R[2, 2] - (R[0, 0] + R[1, 1])
        if xd > 1.0:
            b = 0.5 * np.sqrt(xd); c = 0.25 * (R[0, 1] + R[1, 0]) / b
            d = 0.25 * (R[0, 2] + R[2, 0]) / b; a = 0.25 * (R[2, 1] - R[1, 2]) / b
        elif yd > 1.0:
            c = 0.5 * np.sqrt(yd); b = 0.25 * (R[0, 1] + R[1, 0]) / c
            d = 0.25 * (R[1, 2] + R[2, 1]) / c; a = 0.25 * (R[0, 2] - R[2, 0]) / c
        else:
            d = 0.5 * np.sqrt(zd); b = 0.25 * (R[0, 2] + R[2, 0]) / d
            c = 0.25 * (R[1, 2] + R[2, 1]) / d; a = 0.25 * (R[1, 0] - R[0, 1]) / d
        if a < 0:
            b, c, d = -b, -c, -d
    return b, c, d, qfac, zooms


def save(path, data, affine=None, descrip=b""):
    """Write data (any shape up to 7-D, a dtype of _DTYPES) as a single-file NIfTI-1 image."""
    data = np.asarray(data)
    if data.dtype not in _DTYPES:
        raise ValueError(f"dtype {data.dtype} has no NIfTI-1 code here")
    if not 1 <= data.ndim <= 7:
        raise ValueError("NIfTI-1 holds 1 to 7 dimensions")
    affine = np.eye(4) if affine is None else np.asarray(affine, dtype=np.float64)
    code, bitpix = _DTYPES[data.dtype]
    dim = [data.ndim] + list(data.shape) + [1] * (7 - data.ndim)
    b, c, d, qfac, zooms = _quaternion(affine)
    pixdim = [qfac, zooms[0], zooms[1], zooms[2]] + [1.0] * 4
    h = {"sizeof_hdr": 348, "data_type": b"", "db_name": b"", "extents": 0, "session_error": 0,
         "regular": b"r", "dim_info": 0, "dim": dim, "intent_p1": 0.0, "intent_p2": 0.0,
         "intent_p3": 0.0, "intent_code": 0, "datatype": code, "bitpix": bitpix,
         "slice_start": 0, "pixdim": pixdim, "vox_offset": 352.0, "scl_slope": float("nan"),
         "scl_inter": float("nan"), "slice_end": 0, "slice_code": 0, "xyzt_units": 0,
         "cal_max": 0.0, "cal_min": 0.0, "slice_duration": 0.0, "toffset": 0.0, "glmax": 0,
         "glmin": 0, "descrip": descrip, "aux_file": b"", "qform_code": 0, "sform_code": 2,
         "quatern_b": b, "quatern_c": c, "quatern_d": d, "qoffset_x": affine[0, 3],
         "qoffset_y": affine[1, 3], "qoffset_z": affine[2, 3], "srow_x": list(affine[0]),
         "srow_y": list(affine[1]), "srow_z": list(affine[2]), "intent_name": b"",
         "magic": b"n+1\x00"}
    vals = []
    for name, fmt in _FIELDS:
        v = h[name]
        vals.extend(v if isinstance(v, list) else [v])
    hdr = struct.pack(_FMT, *vals)
    with open(os.fspath(path), "wb") as f:
        f.write(hdr)
        f.write(b"\x00\x00\x00\x00")   # extension flag: none
        f.write(np.asarray(data, order="F").astype(data.dtype.newbyteorder("<"), copy=False)
                .tobytes(order="F"))


def load(path):
    """(data, affine, header dict) of a single-file little-endian NIfTI-1 image."""
    with open(os.fspath(path), "rb") as f:
        buf = f.read()
    if len(buf) < 352:
        raise ValueError("not a NIfTI-1 file (too short)")
    raw = struct.unpack_from(_FMT, buf, 0)
    h, i = {}, 0
    for name, fmt in _FIELDS:
        n = int(fmt[:-1]) if fmt[:-1].isdigit() and fmt[-1] != "s" else 1
        h[name] = list(raw[i:i + n]) if n > 1 else raw[i]
        i += n
    if h["sizeof_hdr"] != 348 or h["magic"] not in (b"n+1\x00", b"ni1\x00"):
        raise ValueError("not a little-endian NIfTI-1 file")
    nd = h["dim"][0]
    shape = tuple(h["dim"][1:1 + nd])
    dt = _CODES[h["datatype"]].newbyteorder("<")
    off = int(h["vox_offset"])
    n = int(np.prod(shape))
    data = np.frombuffer(buf, dtype=dt, count=n, offset=off).reshape(shape, order="F")
    affine = np.eye(4)
    if h["sform_code"] > 0:
        affine[0], affine[1], affine[2] = h["srow_x"], h["srow_y"], h["srow_z"]
    return data, affine, h
