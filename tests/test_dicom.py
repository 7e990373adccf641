"""DICOM ingest: vent_analysis_amd.dicom / .ingest against files written from
the standard's encoding rules.  pydicom is not installed, so the reference loaders
(Vent_Analysis.py:169-223) cannot be run here: parity unpinned -- the checks are round trips of
synthetic studies through all three native transfer syntaxes, the layout the reference produces
(transpose (1, 2, 0), sorted mask slices, float64 mask), the header fields it pulls, and the error
cases.  The GPU test at the end checks that a DICOM-ingested study gives the array path's results."""
import os

import numpy as np
import pytest

from vent_analysis_amd import dicom, ingest
from vent_analysis_amd.synth import synth_volume


def _frame_groups(n, spacing):
    groups = []
    for _ in range(n):
        pm = dicom.Dataset()
        pm.add_new("PixelSpacing", "DS", list(spacing))
        pm.add_new("SliceThickness", "DS", 10.0)
        g = dicom.Dataset()
        g.add_new("PixelMeasuresSequence", "SQ", [pm])
        groups.append(g)
    return groups


def write_xenon(path, vol_u16, vox, ts=dicom.EXPLICIT_LE, undefined=False, groups=True):
    """Multi-frame enhanced-MR-like object: frames = slices, as the scanner export the reference
    transposes back with (1, 2, 0)."""
    R, C, Z = vol_u16.shape
    frames = np.ascontiguousarray(np.transpose(vol_u16, (2, 0, 1)))
    ds = dicom.Dataset()
    ds.add_new("SOPClassUID", "UI", "1.2.840.10008.5.1.4.1.1.4.1")
    ds.add_new("SOPInstanceUID", "UI", "1.2.826.0.1.3680043.9.7433.2.1")
    ds.add_new("StudyDate", "DA", "20240131")
    ds.add_new("StudyTime", "TM", "101500")
    ds.add_new("SeriesTime", "TM", "102000.5")
    ds.add_new("PatientName", "PN", "Doe^Jane")
    ds.add_new("PatientBirthDate", "DA", "19800101")
    ds.add_new("PatientSex", "CS", "F")
    ds.add_new("PatientAge", "AS", "044Y")
    ds.add_new("PatientWeight", "DS", 61.5)
    ds.add_new("SpacingBetweenSlices", "DS", vox[2])
    ds.add_new("SamplesPerPixel", "US", 1)
    ds.add_new("PhotometricInterpretation", "CS", "MONOCHROME2")
    ds.add_new("NumberOfFrames", "IS", Z)
    ds.add_new("Rows", "US", R)
    ds.add_new("Columns", "US", C)
    ds.add_new("BitsAllocated", "US", 16)
    ds.add_new("BitsStored", "US", 16)
    ds.add_new("HighBit", "US", 15)
    ds.add_new("PixelRepresentation", "US", 0)
    if groups:
        ds.add_new("PerFrameFunctionalGroupsSequence", "SQ", _frame_groups(Z, vox[:2]))
    order = ">" if ts == dicom.EXPLICIT_BE else "<"
    ds.add_new("PixelData", "OW", frames.astype(order + "u2").tobytes())
    dicom.write_dataset(path, ds, undefined_length_sequences=undefined, transfer_syntax=ts)


def write_mask_folder(folder, mask_u8, ts=dicom.EXPLICIT_LE):
    os.makedirs(folder, exist_ok=True)
    R, C, Z = mask_u8.shape
    for k in range(Z):
        ds = dicom.Dataset()
        ds.add_new("Rows", "US", R)
        ds.add_new("Columns", "US", C)
        ds.add_new("SamplesPerPixel", "US", 1)
        ds.add_new("BitsAllocated", "US", 8)
        ds.add_new("BitsStored", "US", 8)
        ds.add_new("PixelRepresentation", "US", 0)
        ds.add_new("InstanceNumber", "IS", k + 1)
        ds.add_new("PixelData", "OB", np.ascontiguousarray(mask_u8[:, :, k]).tobytes())
        dicom.write_dataset(os.path.join(folder, f"mask_{k:03d}.dcm"), ds, transfer_syntax=ts)
    with open(os.path.join(folder, "notes.txt"), "w") as f:   # ignored: not .dcm
        f.write("x")


def synth_study(R=24, C=20, Z=5, seed=3):
    x, m = synth_volume(R, C, Z, seed)
    return np.clip(np.rint(x * 10), 0, 65535).astype(np.uint16), m.astype(np.uint8)


@pytest.mark.parametrize("ts", [dicom.EXPLICIT_LE, dicom.IMPLICIT_LE, dicom.EXPLICIT_BE])
@pytest.mark.parametrize("undefined", [False, True])
def test_xenon_round_trip(tmp_path, ts, undefined):
    vol, _ = synth_study()
    p = tmp_path / "xe.dcm"
    write_xenon(p, vol, (1.5, 1.5, 10.0), ts=ts, undefined=undefined)
    ds, arr = ingest.open_single_dicom(p)
    assert ds.transfer_syntax == ts
    assert arr.shape == vol.shape and arr.dtype == np.uint16
    assert np.array_equal(arr, vol)
    assert not arr.flags.c_contiguous   # a transposed view, like the reference (:179)
    meta, vox = ingest.header_metadata(ds)
    assert vox == [1.5, 1.5, 10.0]
    assert meta["PatientName"] == "Doe^Jane" and meta["PatientSex"] == "F"
    assert meta["PatientAge"] == "044Y" and meta["StudyDate"] == "20240131"
    assert meta["PatientWeight"] == 61.5 and meta["SeriesTime"] == "102000.5"
    assert meta["PatientSize"] == ""   # absent elements -> '' (:204-206)
    # pydicom-style access the reference uses
    assert ds[0x5200, 0x9230][0]["PixelMeasuresSequence"][0].PixelSpacing == [1.5, 1.5]
    assert ds.Rows == vol.shape[0] and ds["Columns"].value == vol.shape[1]


@pytest.mark.parametrize("ts", [dicom.EXPLICIT_LE, dicom.IMPLICIT_LE])
def test_mask_folder(tmp_path, ts):
    _, mk = synth_study()
    write_mask_folder(tmp_path / "mask", mk, ts=ts)
    ds, mask = ingest.open_dicom_folder(tmp_path / "mask")
    assert mask.dtype == np.float64 and mask.shape == mk.shape
    assert np.array_equal(mask, mk.astype(np.float64))
    assert ds.InstanceNumber == mk.shape[2]   # the last file's dataset, like the reference


def test_load_study_and_batch(tmp_path):
    studies = []
    ref = []
    for s in range(3):
        vol, mk = synth_study(seed=s)
        d = tmp_path / f"s{s}"
        d.mkdir()
        write_xenon(d / "xe.dcm", vol, (2.0, 2.0, 11.5))
        write_mask_folder(d / "mask", mk)
        studies.append((d / "xe.dcm", d / "mask"))
        ref.append((vol, mk))
    st = ingest.load_study(*studies[0])
    assert st.hp.dtype == np.float32 and st.hp.flags.c_contiguous
    assert np.array_equal(st.hp, ref[0][0].astype(np.float32))
    assert np.array_equal(st.mask, ref[0][1]) and st.vox == [2.0, 2.0, 11.5]
    hp, mk, loaded = ingest.load_batch(studies, workers=3)
    assert hp.shape == (3,) + ref[0][0].shape and hp.dtype == np.float32 and mk.dtype == np.uint8
    for b in range(3):
        assert np.array_equal(hp[b], ref[b][0].astype(np.float32))
        assert np.array_equal(mk[b], ref[b][1])
        assert loaded[b].metadata["PatientName"] == "Doe^Jane"


def test_batch_shape_mismatch(tmp_path):
    a, ma = synth_study(24, 20, 5)
    b, mb = synth_study(24, 20, 6)
    for name, v, m in (("a", a, ma), ("b", b, mb)):
        (tmp_path / name).mkdir()
        write_xenon(tmp_path / name / "xe.dcm", v, (1.5, 1.5, 10.0))
        write_mask_folder(tmp_path / name / "mask", m)
    with pytest.raises(ValueError, match="batch shape"):
        ingest.load_batch([(tmp_path / n / "xe.dcm", tmp_path / n / "mask") for n in "ab"])
    with pytest.raises(ValueError, match="mask shape"):
        ingest.load_study(tmp_path / "a" / "xe.dcm", tmp_path / "b" / "mask")


def test_errors_and_pixel_variants(tmp_path):
    p = tmp_path / "raw.bin"
    p.write_bytes(b"\x00" * 64)
    with pytest.raises(dicom.InvalidDicomError):
        dicom.dcmread(p)
    # header without PixelSpacing -> ValueError (the reference prompts on stdin)
    vol, _ = synth_study()
    write_xenon(tmp_path / "nogroups.dcm", vol, (1.5, 1.5, 10.0), groups=False)
    with pytest.raises(ValueError, match="PixelSpacing"):
        ingest.header_metadata(dicom.dcmread(tmp_path / "nogroups.dcm"))
    # ... but the patient/study fields are still available (the reference stores them first)
    info = ingest.header_info(dicom.dcmread(tmp_path / "nogroups.dcm"))
    assert info["PatientName"] == "Doe^Jane" and info["StudyDate"] == "20240131"
    # signed 12-bit stored in 16: sign extension like pydicom's numpy handler
    ds = dicom.Dataset()
    vals = np.array([[0x0FFF, 0x0800], [0x07FF, 0x0001]], np.uint16)   # -1, -2048, 2047, 1
    for kw, vr, v in (("Rows", "US", 2), ("Columns", "US", 2), ("BitsAllocated", "US", 16),
                      ("BitsStored", "US", 12), ("PixelRepresentation", "US", 1)):
        ds.add_new(kw, vr, v)
    ds.add_new("PixelData", "OW", vals.tobytes())
    dicom.write_dataset(tmp_path / "s12.dcm", ds)
    arr = dicom.dcmread(tmp_path / "s12.dcm").pixel_array
    assert arr.dtype == np.int16 and arr.tolist() == [[-1, -2048], [2047, 1]]
    # single frame without NumberOfFrames -> 2-D; the reference's 3-axis transpose then fails
    with pytest.raises(ValueError):
        ingest.open_single_dicom(tmp_path / "s12.dcm")
    # empty mask folder
    (tmp_path / "empty").mkdir()
    with pytest.raises(IndexError):
        ingest.open_dicom_folder(tmp_path / "empty")


def test_vent_analysis_ctor_from_dicom(tmp_path):
    """Constructor with xenon_path / mask_path (Vent_Analysis.py:111-136): image, mask, vox and
    metadata from the files.  The mask border needs the GPU; without one the constructor reports
    the failure and keeps the mask, like the reference's try/except."""
    from vent_analysis_amd import Vent_Analysis
    vol, mk = synth_study()
    write_xenon(tmp_path / "xe.dcm", vol, (1.5, 1.5, 10.0))
    write_mask_folder(tmp_path / "mask", mk)
    va = Vent_Analysis(xenon_path=str(tmp_path / "xe.dcm"), mask_path=str(tmp_path / "mask"))
    assert np.array_equal(va.HPvent, vol) and np.array_equal(va.mask, mk.astype(np.float64))
    assert va.vox == [1.5, 1.5, 10.0] and va.metadata["PatientName"] == "Doe^Jane"
    lv = np.sum(mk == 1) * np.prod(np.divide([1.5, 1.5, 10.0], 10)) / 1000
    assert va.metadata["LungVolume"] == lv


@pytest.mark.gpu
def test_dicom_study_matches_array_path(tmp_path):
    from vent_analysis_amd import Vent_Analysis
    vol, mk = synth_study(48, 40, 8, seed=5)
    write_xenon(tmp_path / "xe.dcm", vol, (1.5, 1.5, 10.0))
    write_mask_folder(tmp_path / "mask", mk)
    a = Vent_Analysis(xenon_path=str(tmp_path / "xe.dcm"), mask_path=str(tmp_path / "mask"))
    b = Vent_Analysis(xenon_array=vol, mask_array=mk.astype(np.float64), vox=[1.5, 1.5, 10.0])
    assert np.array_equal(a.mask_border, b.mask_border)
    a.calculate_VDP()
    b.calculate_VDP()
    assert np.array_equal(a.N4HPvent, b.N4HPvent)
    assert np.array_equal(a.defectArray, b.defectArray)
    for k in ("VDP", "VDP_lb", "VDP_km", "SNR", "LungVolume", "DefectVolume"):
        assert a.metadata[k] == b.metadata[k], k


def test_load_study_mask_validation(tmp_path):
    """Non-binary or empty masks raise instead of silently becoming empty studies."""
    vol, mk = synth_study(seed=4)
    write_xenon(tmp_path / "xe.dcm", vol, (2.0, 2.0, 11.5))
    write_mask_folder(tmp_path / "m255", (mk * 255).astype(mk.dtype))
    with pytest.raises(ValueError, match="0/1"):
        ingest.load_study(tmp_path / "xe.dcm", tmp_path / "m255")
    write_mask_folder(tmp_path / "m0", np.zeros_like(mk))
    with pytest.raises(ValueError, match="no mask voxels"):
        ingest.load_study(tmp_path / "xe.dcm", tmp_path / "m0")
