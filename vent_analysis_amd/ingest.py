"""DICOM ingest for batch runs: study files -> contiguous device-ready arrays.

Restates the reference's loaders (Vent_Analysis.py:169-223) on top of ``vent_analysis_amd.dicom``:

* ``open_single_dicom``  -- :169-181: ``pixel_array`` transposed (1, 2, 0), i.e. a multi-frame
  (frames, rows, cols) object becomes (rows, cols, frames); the reference keeps the transposed
  *view*; batch loading makes it contiguous once (the C-ABI needs C-order).
* ``open_dicom_folder``  -- :184-196: every ``*.dcm`` of the folder in sorted name order, one
  slice each, stacked on the last axis as float64 (the reference's ``np.zeros`` dtype).
* ``header_info`` / ``header_vox`` / ``header_metadata`` -- :198-223: the patient/study elements
  (missing ones -> ''), and vox = [PixelSpacing of the first per-frame functional group that has
  one, SpacingBetweenSlices].  Where the reference prompts on stdin for a missing spacing
  ``header_vox`` raises ValueError instead; the info elements are read separately first, as the
  reference stores them before it looks at the spacing (:200-206).
* ``load_study`` / ``load_batch`` -- one study or many into the (B, R, C, Z) float32 / uint8
  arrays ``_lib.Batch.upload`` takes, plus vox and the metadata; files are parsed on a thread pool.

The mask must be binary (0/1) and non-empty; it is handed to the device as uint8.  Other label
values raise ValueError rather than silently becoming an empty study: the reference's chain
selects mask > 0 (:245) while N4 uses MaskLabel 1, so a 0/255 mask has no N4 voxels.  The class
path (``Vent_Analysis._mask_value``) implements that case per study (N4 := identity, maps scaled
by the mask value); a batch runs one N4 setting for all its studies, so it takes 0/1 masks only.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from .dicom import dcmread

__all__ = ["open_single_dicom", "open_dicom_folder", "header_info", "header_vox",
           "header_metadata", "Study", "load_study", "load_batch"]

INFO_ELEMENTS = ['PatientName', 'PatientAge', 'PatientBirthDate', 'PatientSize', 'PatientWeight',
                 'PatientSex', 'StudyDate', 'StudyTime', 'SeriesTime']


def open_single_dicom(path):
    """(ds, pixel_array transposed to (rows, cols, frames)) -- Vent_Analysis.py:169-181."""
    ds = dcmread(path)
    return ds, np.transpose(ds.pixel_array, (1, 2, 0))


def mask_files(folder):
    return [f for f in sorted(os.listdir(folder)) if f.endswith('.dcm')]


def open_dicom_folder(folder, workers=8):
    """(last ds, float64 mask (rows, cols, n_files)) -- Vent_Analysis.py:184-196."""
    files = mask_files(folder)
    if not files:
        raise IndexError(f"no .dcm files in {folder}")   # dcm_filelist[0] in the reference
    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        dss = list(ex.map(lambda f: dcmread(os.path.join(folder, f)), files))
    first = dss[0].pixel_array
    mask = np.zeros((first.shape[0], first.shape[1], len(files)))
    for k, ds in enumerate(dss):
        mask[:, :, k] = ds.pixel_array
    return dss[-1], mask


def header_info(ds):
    """The patient/study elements of the xenon header (absent ones -> '') -- Vent_Analysis.py:200-206."""
    meta = {}
    for elem in INFO_ELEMENTS:
        try:
            meta[elem] = ds[elem].value
        except KeyError:
            meta[elem] = ''
    return meta


def header_vox(ds):
    """vox = [dx, dy, dz] from the xenon header -- Vent_Analysis.py:207-223 (ValueError where the
    reference prompts on stdin)."""
    spacing = None
    try:
        groups = ds[0x5200, 0x9230]
        for k in range(min(100, len(groups))):   # the reference tries items 0..99
            try:
                spacing = groups[k]['PixelMeasuresSequence'][0].PixelSpacing
                break
            except (KeyError, IndexError, AttributeError):
                continue
    except KeyError:
        pass
    if spacing is None:
        raise ValueError("PixelSpacing not in the per-frame functional groups "
                         "(the reference prompts for it on stdin, Vent_Analysis.py:213-215)")
    try:
        dz = float(ds.SpacingBetweenSlices)
    except AttributeError:
        raise ValueError("SpacingBetweenSlices missing (the reference prompts for it on stdin, "
                         "Vent_Analysis.py:219-221)") from None
    return [float(spacing[0]), float(spacing[1]), dz]


def header_metadata(ds):
    """(metadata dict, vox) from the xenon header -- Vent_Analysis.py:198-223."""
    return header_info(ds), header_vox(ds)


def binary_mask(mask, what="mask"):
    """uint8 0/1 copy of a binary mask; ValueError for other labels or an empty mask."""
    m = np.asarray(mask)
    u8 = (m != 0).astype(np.uint8)
    if not np.array_equal(u8, m):
        raise ValueError(f"{what}: labels other than 0/1 (the GPU path implements binary masks; "
                         "binarise before loading)")
    if not u8.any():
        raise ValueError(f"{what}: no mask voxels")
    return np.ascontiguousarray(u8)


@dataclass
class Study:
    hp: np.ndarray            # float32 (R, C, Z), C-contiguous
    mask: np.ndarray          # uint8 (R, C, Z), mask == 1
    vox: list
    metadata: dict = field(default_factory=dict)
    path: str = ''


def load_study(xenon_path, mask_folder, workers=8):
    """One study: xenon DICOM file + mask folder -> contiguous float32 / uint8 (R, C, Z) + vox."""
    ds, hp = open_single_dicom(xenon_path)
    meta, vox = header_metadata(ds)
    _, mask = open_dicom_folder(mask_folder, workers=workers)
    if mask.shape != hp.shape:
        raise ValueError(f"{xenon_path}: mask shape {mask.shape} != image shape {hp.shape}")
    return Study(hp=np.ascontiguousarray(hp, dtype=np.float32),
                 mask=binary_mask(mask, f"{mask_folder}"), vox=vox, metadata=meta,
                 path=os.fspath(xenon_path))


def load_batch(studies, workers=8):
    """[(xenon_path, mask_folder), ...] -> (hp [B,R,C,Z] f32, mask [B,R,C,Z] u8, [Study]) for
    ``_lib.Batch.upload``.  Studies are parsed in parallel; all must share one (R, C, Z)."""
    studies = list(studies)
    if not studies:
        raise ValueError("load_batch: no studies")
    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        loaded = list(ex.map(lambda sm: load_study(sm[0], sm[1], workers=1), studies))
    shape = loaded[0].hp.shape
    for s in loaded:
        if s.hp.shape != shape:
            raise ValueError(f"load_batch: {s.path} has shape {s.hp.shape}, batch shape {shape}")
    from ._lib import empty_aligned   # page-aligned: _lib.Pipe DMAs whole chunks in place
    hp = empty_aligned((len(loaded),) + shape, np.float32)
    mk = empty_aligned((len(loaded),) + shape, np.uint8)
    for b, s in enumerate(loaded):
        hp[b] = s.hp
        mk[b] = s.mask
    return hp, mk, loaded
