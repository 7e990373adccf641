"""Pickle compatibility of the drop-in class (Vent_Analysis.py:542-559, :153-164).

CPU only: a study restored from a pickle dict needs no GPU call (the constructor computes the mask
border only for a mask_array / mask_path), so these run without libventhip.so compute.

The reference pickles ``vars(self)`` minus unpicklable attributes (``pickleMe``, :542-553) and
restores by ``setattr`` over the dict (``unPickleMe``, :556-559); the GUI's "Load Pickle" path
builds the class from ``pickle_path`` (:839).  A reference pickle is a plain dict of numpy arrays,
strings, lists and the metadata dict, so these tests build such a dict with the reference's
attribute names and dtypes and check both directions.
"""
import pickle

import numpy as np
import pytest

from vent_analysis_amd import Vent_Analysis
from vent_analysis_amd.synth import synth_volume


def _reference_style_dict():
    X, M = synth_volume(32, 40, 6, 3)
    M = M.astype(np.float64)                       # openDICOMfolder builds float64 masks (:191)
    d = {
        "version": "241007_vent",
        "HPvent": X, "mask": M, "mask_border": np.zeros_like(M), "proton": "",
        "N4HPvent": X.astype(np.float32), "defectArray": (X < 50).astype(np.float64) * M,
        "defectBorder": np.zeros(M.shape, bool), "defectArrayLB": np.ones_like(M) * M,
        "CIarray": np.zeros_like(M), "vox": [1.5, 1.5, 10.0], "ds": "", "twix": "",
        "raw_k": "", "raw_HPvent": "",
        "metadata": {"fileName": "study.dcm", "PatientName": "anon", "VDP": 7.25, "VDP_lb": 3.5,
                     "VDP_km": "", "SNR": np.float32(30.5), "LungVolume": 0.1,
                     "DefectVolume": 0.01, "CI": 22.5},
    }
    return d


def test_restore_from_reference_style_pickle(tmp_path):
    d = _reference_style_dict()
    p = tmp_path / "ref.pkl"
    with open(p, "wb") as f:
        pickle.dump(d, f)
    v = Vent_Analysis(pickle_path=str(p))
    for k, val in d.items():
        got = getattr(v, k)
        if isinstance(val, np.ndarray):
            assert got.dtype == val.dtype and np.array_equal(got, val), k
        elif k != "metadata":
            assert got == val, k
    # the metadata dict is restored as a whole (unPickleMe setattr), then LungVolume recomputed
    # from mask and vox exactly as the reference constructor does (:166)
    assert v.metadata["VDP"] == 7.25 and v.metadata["CI"] == 22.5
    exp = np.sum(d["mask"] == 1) * np.prod(np.divide(d["vox"], 10)) / 1000
    assert v.metadata["LungVolume"] == exp


def test_pickle_round_trip_keeps_attribute_set(tmp_path):
    d = _reference_style_dict()
    v = Vent_Analysis(pickle_dict=d)
    v.n4_iterations = [19, 4, 2, 2]
    p = tmp_path / "out.pkl"
    v.pickleMe(str(p))
    with open(p, "rb") as f:
        back = pickle.load(f)
    assert set(d) <= set(back)                      # every reference attribute survives
    assert set(back) == set(vars(v))                # and exactly the picklable attribute set
    for k in d:
        if isinstance(d[k], np.ndarray):
            assert np.array_equal(back[k], d[k]) and back[k].dtype == d[k].dtype, k
    w = Vent_Analysis(pickle_dict=back)
    assert w.vox == d["vox"] and np.array_equal(w.defectArray, d["defectArray"])


def test_pickle_skips_unpicklable_attributes(tmp_path, capsys):
    v = Vent_Analysis(pickle_dict=_reference_style_dict())
    v.handle = lambda: None                          # e.g. a GUI callback left on the object
    p = tmp_path / "skip.pkl"
    v.pickleMe(str(p))
    assert "Skipping non-picklable attribute: handle" in capsys.readouterr().out
    with open(p, "rb") as f:
        assert "handle" not in pickle.load(f)


def test_build4DdataArray_channel_layout():
    """Vent_Analysis.py:292-313: channels proton, HPvent, mask, N4HPvent, defectArray, CIarray;
    a missing channel is skipped with a message (proton is '' here)."""
    d = _reference_style_dict()
    v = Vent_Analysis(pickle_dict=d)
    a = v.build4DdataArray()
    assert a.shape == d["HPvent"].shape + (6,) and a.dtype == np.float32
    assert np.array_equal(a[..., 1], d["HPvent"].astype(np.float32))
    assert np.array_equal(a[..., 2], d["mask"].astype(np.float32))
    assert np.array_equal(a[..., 4], d["defectArray"].astype(np.float32))
    assert not a[..., 0].any()


def test_missing_pickle_path_is_reported_not_raised(tmp_path, capsys):
    """The reference ctor swallows a failed pickle load with a message (:156-161); with no mask
    the LungVolume line then raises AttributeError exactly like the reference (:166)."""
    with pytest.raises(AttributeError):
        Vent_Analysis(pickle_path=str(tmp_path / "nope.pkl"))
    assert "Opening Pickle from path and building arrays failed" in capsys.readouterr().out
