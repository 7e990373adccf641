"""4-D NIfTI export (Vent_Analysis.py:273-313).  nibabel is not installed, so
the writer is checked against the NIfTI-1 layout itself (parity unpinned): header fields, the
352-byte data offset, Fortran voxel order, and round trips."""
import struct

import numpy as np
import pytest

from vent_analysis_amd import nifti


def test_header_layout_and_fortran_order(tmp_path):
    a = np.arange(2 * 3 * 4 * 6, dtype=np.float32).reshape(2, 3, 4, 6)
    p = tmp_path / "x.nii"
    nifti.save(p, a, affine=np.eye(4))
    buf = p.read_bytes()
    assert len(buf) == 352 + a.nbytes
    assert struct.unpack_from("<i", buf, 0)[0] == 348
    assert struct.unpack_from("<8h", buf, 40) == (4, 2, 3, 4, 6, 1, 1, 1)
    assert struct.unpack_from("<hh", buf, 70) == (16, 32)          # datatype float32, bitpix
    assert struct.unpack_from("<f", buf, 108)[0] == 352.0          # vox_offset
    assert np.isnan(struct.unpack_from("<f", buf, 112)[0])         # scl_slope: no scaling
    assert struct.unpack_from("<hh", buf, 252) == (0, 2)           # qform_code, sform_code
    assert struct.unpack_from("<12f", buf, 280) == (1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0)
    assert buf[344:348] == b"n+1\x00"
    vox = np.frombuffer(buf, np.float32, offset=352)
    assert np.array_equal(vox, a.ravel(order="F"))                # first axis fastest
    d, aff, h = nifti.load(p)
    assert np.array_equal(d, a) and np.array_equal(aff, np.eye(4)) and h["pixdim"][:4] == [1, 1, 1, 1]


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.float32, np.float64])
def test_round_trip_dtypes(tmp_path, dtype):
    rng = np.random.default_rng(1)
    a = (rng.random((5, 4, 3)) * 100).astype(dtype)
    aff = np.diag([1.5, 1.5, 10.0, 1.0])
    aff[:3, 3] = (-10.0, 4.0, 2.5)
    nifti.save(tmp_path / "y.nii", a, affine=aff)
    d, aff2, h = nifti.load(tmp_path / "y.nii")
    assert d.dtype == np.dtype(dtype) and np.array_equal(d, a)
    assert np.allclose(aff2, aff) and np.allclose(h["pixdim"][1:4], [1.5, 1.5, 10.0])


def test_qform_quaternion_of_a_rotation(tmp_path):
    aff = np.array([[0.0, -2.0, 0.0, 1.0], [2.0, 0.0, 0.0, 2.0], [0.0, 0.0, 3.0, 3.0],
                    [0.0, 0.0, 0.0, 1.0]])   # 90 degrees about z, zooms (2, 2, 3)
    nifti.save(tmp_path / "r.nii", np.zeros((2, 2, 2), np.float32), affine=aff)
    _, _, h = nifti.load(tmp_path / "r.nii")
    b, c, d = h["quatern_b"], h["quatern_c"], h["quatern_d"]
    a = np.sqrt(max(0.0, 1 - b * b - c * c - d * d))
    R = np.array([[a*a + b*b - c*c - d*d, 2*(b*c - a*d), 2*(b*d + a*c)],
                  [2*(b*c + a*d), a*a + c*c - b*b - d*d, 2*(c*d - a*b)],
                  [2*(b*d - a*c), 2*(c*d + a*b), a*a + d*d - c*c - b*b]])
    assert np.allclose(R * np.array(h["pixdim"][1:4]), aff[:3, :3], atol=1e-6)


def test_export_nifti_from_class(tmp_path):
    from vent_analysis_amd import Vent_Analysis
    va = Vent_Analysis.__new__(Vent_Analysis)   # attributes only: no device work
    va.metadata = {'PatientName': 'Doe^Jane'}
    va.HPvent = np.full((4, 3, 2), 7, np.float32)
    va.mask = np.ones((4, 3, 2))
    va.proton = ''
    va.N4HPvent = np.full((4, 3, 2), 2, np.float32)
    va.defectArray = np.zeros((4, 3, 2))
    va.CIarray = ''
    va.exportNifti(str(tmp_path))
    d, aff, _ = nifti.load(tmp_path / "Doe_Jane_dataArray.nii")
    assert d.shape == (4, 3, 2, 6) and d.dtype == np.float32
    assert np.array_equal(d, va.build4DdataArray())
    assert np.all(d[..., 1] == 7) and np.all(d[..., 3] == 2) and np.all(d[..., 0] == 0)
