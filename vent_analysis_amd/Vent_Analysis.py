"""Vent_Analysis -- drop-in for the reference class (Vent_Analysis.py:26-577), GPU hot path.

Keeps the constructor keywords, method names, attribute names/dtypes and metadata keys the GUI
reads (Vent_Analysis.py:724-781, 839-1004), so it can replace ``from Vent_Analysis import
Vent_Analysis``.  The voxel work -- N4, SNR, the mean-anchored / linear-binning / k-means VDP
chain, defect/mask borders and the cluster index -- runs in libventhip.so on an MI355X
(include/vent_hip.h).  Host code only moves arrays, casts dtypes and fills the metadata dict.
There is no CPU fallback: a missing library raises ImportError on first use.

Additions (backward compatible): a ``vox=`` constructor keyword (the reference's array-only
constructor crashes at Vent_Analysis.py:166 because vox is '' -- pass vox to avoid it) and
``metadata['VDP_km']`` is now filled (the reference leaves it '', :259-261; build-defined k-means).
"""
from __future__ import annotations

import os
import pickle

import numpy as np

from . import CI
from . import _lib
from . import ingest
from . import nifti

__all__ = ["Vent_Analysis"]


def _binary_u8(A, what):
    a = np.asarray(A)
    if a.dtype == np.uint8 and a.max(initial=0) <= 1:
        return np.ascontiguousarray(a)
    u8 = (a != 0).astype(np.uint8)
    if not np.array_equal(u8, a):
        raise ValueError(f"{what} must be binary (0/1); the GPU path implements the reference's "
                         "behaviour for binary masks only")
    return u8


def _mask_value(A, what='mask'):
    """(mask != 0 as uint8 0/1, v) for a mask whose nonzero voxels all hold one positive value v
    (0/1, 0/255, ...: what mask DICOM folders hold).  The reference works on any such mask:
    ``mask > 0`` selects the signal (Vent_Analysis.py:245, :340), the defect and LB maps are
    multiplied by the mask (:249, :256) and VDP divides by ``np.sum(mask)`` (:251, :257), so v
    scales the maps and cancels in VDP.  Masks with several nonzero values (a median over mixed
    values) or negative values raise ValueError."""
    a = np.asarray(A)
    if a.dtype == np.uint8 and a.max(initial=0) <= 1:
        return np.ascontiguousarray(a), 1
    nz = a != 0
    vals = np.unique(a[nz]) if nz.any() else np.array([1])
    if vals.size != 1 or not vals[0] > 0:
        raise ValueError(f"{what}: the GPU path implements the reference's behaviour for masks "
                         f"whose nonzero voxels share one positive value (got {vals[:4]}...)")
    v = vals[0].item()
    return nz.astype(np.uint8), (1 if v == 1 else v)


def _n4_label(v):
    """Whether N4 sees the mask voxels: the reference casts the mask to float32 and then to
    sitk.UInt8 (Vent_Analysis.py:323-327, truncation) and SimpleITK's N4 uses label 1 only
    (MaskLabel 1, UseMaskLabel true: SURVEY A.2).  A 0/255 mask therefore has no N4 voxels."""
    return int(np.float32(v)) == 1


class Vent_Analysis:
    """Complete VDP analysis: N4 bias correction, normalisation, defect maps, VDPs, CI.
    See the reference docstring (Vent_Analysis.py:27-57) for the attribute list."""

    def __init__(self, xenon_path=None, mask_path=None, proton_path=None, xenon_array=None,
                 mask_array=None, proton_array=None, pickle_dict=None, pickle_path=None,
                 vox=None, device=0):
        self.version = '241007_vent'
        self.device = device
        self.proton = ''
        self.N4HPvent = ''
        self.defectArray = ''
        self.CIarray = ''
        self.vox = ''
        self.ds = ''
        self.twix = ''
        self.raw_k = ''
        self.raw_HPvent = ''
        self.metadata = {'fileName': '', 'PatientName': '', 'PatientAge': '',
                         'PatientBirthDate': '', 'PatientSex': '', 'Disease': '', 'StudyDate': '',
                         'SeriesTime': '', 'DE': '', 'SNR': '', 'VDP': '', 'VDP_lb': '',
                         'VDP_km': '', 'LungVolume': '', 'DefectVolume': '', 'CI': '',
                         'FEV1': '', 'FVC': '', 'visit': '', 'IRB': '', 'treatment': '',
                         'analysisUser': '', 'notes': ''}

        if xenon_array is not None:
            print(f'\033[34mXenon array provided: {xenon_array.shape}\033[37m')
            self.HPvent = xenon_array
        if xenon_path is not None:
            try:
                print('\033[34mXenon DICOM path provided. Opening DICOM...\033[37m')
                self.ds, self.HPvent = self.openSingleDICOM(xenon_path)
            except Exception:
                print('\033[31mOpening Xenon DICOM failed...\033[37m')
            try:
                print('\033[34mPulling Xenon DICOM Header\033[37m')
                self.pullDICOMHeader()
            except Exception:
                print('\033[31mPulling Xenon DICOM Header failed...\033[37m')
        if mask_array is not None:
            print(f'\033[34mMask array provided: {mask_array.shape}\033[37m')
            self.mask = mask_array
            self.mask_border = self.calculateBorder(self.mask)
        if mask_path is not None:
            try:
                print('\033[34mLoading Mask and calculating border\033[37m')
                _, self.mask = self.openDICOMfolder(mask_path)
                self.mask_border = self.calculateBorder(self.mask)
            except Exception:
                print('\033[31mLoading Mask and calculating border failed...\033[37m')
        if proton_array is not None:
            print(f'\033[34mProton array provided: {proton_array.shape}\033[37m')
            self.proton = proton_array
        if proton_path is not None:
            try:
                print('\033[34mProton DICOM Path provided. Opening...\033[37m')
                self.proton_ds, self.proton = self.openSingleDICOM(proton_path)
            except Exception:
                print('\033[31mOpening Proton DICOM failed...\033[37m')
        if pickle_path is not None:
            print(f'\033[34mPickle path provided: {pickle_path}. Loading...\033[37m')
            try:
                with open(pickle_path, 'rb') as file:
                    pickle_dict = pickle.load(file)   # the user's own study pickle (:153-155)
                print('\033[32mPickle file successfully loaded.\033[37m')
            except Exception:
                print('\033[31mOpening Pickle from path and building arrays failed...\033[37m')
        if pickle_dict is not None:
            self.unPickleMe(pickle_dict)
        if vox is not None:
            self.vox = [float(v) for v in vox]
        self.metadata['LungVolume'] = np.sum(self.mask == 1) * np.prod(np.divide(self.vox, 10)) / 1000

    # ---- DICOM ingest (vent_analysis_amd.ingest, no pydicom needed) -------
    def openSingleDICOM(self, dicom_path):
        """Vent_Analysis.py:169-181: (dataset, pixel_array transposed to (rows, cols, frames))."""
        ds, arr = ingest.open_single_dicom(dicom_path)
        print(f'\033[32mI opened a DICOM of shape {arr.shape}\033[37m')
        return ds, arr

    def openDICOMfolder(self, maskFolder):
        """Vent_Analysis.py:184-196: the folder's .dcm slices (sorted) stacked as float64."""
        ds, mask = ingest.open_dicom_folder(maskFolder)
        print(f'\033[32mI built a mask of shape {mask.shape}\033[37m')
        return ds, mask

    def pullDICOMHeader(self):
        """Vent_Analysis.py:198-223: patient/study elements into metadata, vox from the header."""
        self.metadata.update(ingest.header_info(self.ds))   # stored before the spacing lookup
        self.vox = ingest.header_vox(self.ds)
        self.metadata['LungVolume'] = np.sum(self.mask == 1) * np.prod(np.divide(self.vox, 10)) / 1000

    # ---- hot path ---------------------------------------------------------------------------
    def calculateBorder(self, A):
        """Vent_Analysis.py:225-231 on the GPU: per slice, np.gradient != 0 along rows or cols.
        Returns float64 0/1.  Equality is all that matters, so any array with <= 256 distinct
        values is exact (values are replaced by their rank)."""
        a = np.asarray(A)
        if a.dtype == np.bool_ or (a.size and a.min() >= 0 and a.max() <= 1 and np.all(a == np.round(a))):
            u8 = np.ascontiguousarray(a, dtype=np.uint8)
        else:
            uniq, inv = np.unique(a, return_inverse=True)
            if uniq.size > 256:
                raise ValueError("calculateBorder: more than 256 distinct values")
            u8 = inv.reshape(a.shape).astype(np.uint8)
        return _lib.border(u8, device=self.device)[0].astype(np.float64)

    def normalize(self, x):
        if (np.max(x) - np.min(x)) == 0:
            return x
        return (x - np.min(x)) / (np.max(x) - np.min(x))

    def _n4_overridden(self):
        return 'N4_bias_correction' in self.__dict__

    def calculate_VDP(self, thresh=0.6):
        """Vent_Analysis.py:239-263 as one GPU pipeline: SNR, N4, sorted masked list -> numpy-order
        mean anchor, threshold + 3x3 median + border, 99th-pct linear binning, k-means, volumes.

        A mask of one nonzero value v != 1 (e.g. 0/255) runs the kernels on mask != 0 and scales
        the maps by v as ``* self.mask`` does; VDP, VDP_lb and DefectVolume then follow the
        reference's expressions on the scaled maps (v cancels in VDP; ``== 1`` tests find no
        voxel for v = 255).  Such a mask has no voxel of N4's label 1 (_n4_label), and ITK's N4
        on an empty label set leaves the image as it is (no histogram, an all-zero B-spline fit,
        a NaN convergence measure that ends every level after one iteration): N4HPvent = HPvent,
        parity unpinned (SimpleITK absent)."""
        mask_u8, v = _mask_value(self.mask)
        hp = np.asarray(self.HPvent)
        vox = np.asarray(self.vox, dtype=np.float64)
        if self._n4_overridden():
            # a caller-supplied N4 (e.g. identity): GPU chain on its output
            self.metadata['SNR'] = self.calculate_SNR(self.HPvent, self.mask)
            self.N4HPvent = self.N4_bias_correction(self.HPvent, self.mask)
            d, bo, lb, res = _lib.vdp(self.N4HPvent, mask_u8, vox, hp=None, thresh=thresh,
                                      device=self.device)
        else:
            do_n4 = _n4_label(v)
            with _lib.pooled_batch(*hp.shape, 1, device=self.device) as B:   # reused across calls
                B.upload(hp.astype(np.float32)[None], mask_u8[None])
                B.run(B.options(do_n4=do_n4, thresh=thresh, vox=vox))
                n4, d, bo, lb, res = B.download(n4=True)
            if res[0].n_mask == 0:   # sorted([])[int(0 * 0.99)] in the reference (:245, :255)
                raise IndexError("calculate_VDP: empty mask (list index out of range)")
            self.N4HPvent = n4[0]
            self.metadata['SNR'] = self._snr_dtype(res[0].snr, hp)
        r = res[0]
        msum = np.sum(self.mask)
        self.defectBorder = bo[0] == 1
        self.defectArrayLB = lb[0].astype(np.float64) * np.asarray(self.mask)
        if v == 1:
            self.defectArray = d[0].astype(np.float64)
            self.metadata['VDP'] = 100 * np.float64(r.n_defect) / msum
            self.metadata['DefectVolume'] = r.n_defect * np.prod(np.divide(self.vox, 10)) / 1000
            self.metadata['VDP_lb'] = 100 * np.float64(r.n_lb12) / msum
        else:   # the reference's expressions on the v-scaled maps (:249-257)
            self.defectArray = d[0].astype(np.float64) * v
            self.metadata['VDP'] = 100 * np.sum(self.defectArray) / msum
            self.metadata['DefectVolume'] = (np.sum(self.defectArray == 1)
                                             * np.prod(np.divide(self.vox, 10)) / 1000)
            self.metadata['VDP_lb'] = 100 * np.sum((self.defectArrayLB == 1) * 1
                                                   + (self.defectArrayLB == 2) * 1) / msum
        self.metadata['VDP_km'] = 100 * np.float64(r.n_km0) / np.float64(r.n_mask)
        self.n4_iterations = list(r.n4_iters)[:4]
        print('\033[32mcalculate_VDP ran successfully\033[37m')

    @staticmethod
    def _snr_dtype(v, A):
        dt = np.asarray(A).dtype
        if dt == np.float32 or dt == np.float16:
            return np.float32(v)
        return np.float64(v)

    def calculate_CI(self):
        """Vent_Analysis.py:265-271: CIarray + 95th-percentile CI, one GPU pass."""
        self.CIarray, ci = CI.calculate_CI_with_index(self.defectArray, self.vox, device=self.device)
        self.metadata['CI'] = ci
        print(f"Calculated CI: {self.metadata['CI']}")

    def N4_bias_correction(self, HPvent, mask):
        """Vent_Analysis.py:316-334: N4 with the SimpleITK 2.3.1 defaults, on the GPU.
        Returns float32 like sitk.GetArrayFromImage."""
        m = np.asarray(mask).astype(np.float32)
        m = ((m >= 1) & (m < 2)).astype(np.uint8)   # sitk.Cast(..., UInt8) == label 1 (:323-327)
        if not m.any():
            # Empty label set (e.g. a 0/255 mask): no voxel to fit.  Returned as the image unchanged,
            # which is what ITK's N4 computes when its fit has no points (an all-zero field).
            # PARITY UNPINNED: SimpleITK is absent, so neither that output nor ITK's iteration
            # counts on an empty label set are checked against the reference.  n4_iterations is
            # the sentinel [0, 0, 0, 0] = "N4 not run", not a claim about ITK's counts.
            self.n4_iterations = [0, 0, 0, 0]
            return np.asarray(HPvent, dtype=np.float32).copy()
        out, its, _ = _lib.n4(np.asarray(HPvent, dtype=np.float32), m, device=self.device)
        self.n4_iterations = list(its[0])
        return out[0]

    def calculate_SNR(self, A, FOVbuffer=20, manualNoise=False):
        """Vent_Analysis.py:337-357 on the GPU (noise box from self.mask, FOVbuffer forced to 20
        like the reference).  Returns A's float dtype (float32 for float32 input)."""
        if manualNoise:
            raise UnboundLocalError("cannot access local variable 'noise' (manualNoise branch is "
                                    "empty in the reference, Vent_Analysis.py:353-355)")
        m, _ = _mask_value(self.mask)
        v = _lib.snr(np.asarray(A, dtype=np.float32), m, device=self.device)[0]
        return self._snr_dtype(v, A)

    # ---- persistence / export helpers (format compat, not voxel compute) ---------------------
    def build4DdataArray(self):
        """Vent_Analysis.py:292-313: Proton, HPvent, mask, N4HPvent, defectArray, CIarray."""
        dataArray = np.zeros(tuple(self.HPvent.shape) + (6,), dtype=np.float32)
        dataArray[:, :, :, 1] = self.HPvent
        dataArray[:, :, :, 2] = self.mask
        for ch, name in ((0, 'proton'), (3, 'N4HPvent'), (4, 'defectArray'), (5, 'CIarray')):
            try:
                dataArray[:, :, :, ch] = getattr(self, name)
            except Exception:
                print(f'\033[33m{name} does not exist and was not added to 4D array\033[37m')
        return dataArray

    def cropToData(self, A, border=0, borderSlices=False):
        """Vent_Analysis.py:430-456, including its quirk: the per-axis "non-empty" flags are
        multiplied by the index list, so index 0 never counts as non-empty."""
        fs = np.multiply(np.sum(np.sum(A, axis=0), axis=0) > 0, list(range(0, A.shape[2])))
        fr = np.multiply(np.sum(np.sum(A, axis=1), axis=1) > 0, list(range(0, A.shape[0])))
        fc = np.multiply(np.sum(np.sum(A, axis=2), axis=0) > 0, list(range(0, A.shape[1])))
        slices = [x for x in range(A.shape[2]) if fs[x]]
        rows = [x for x in range(A.shape[0]) if fr[x]]
        cols = [x for x in range(A.shape[1]) if fc[x]]
        if borderSlices:
            s0, s1 = max(slices[0] - border, 0), min(slices[-1] + border + 1, A.shape[2])
        else:
            s0, s1 = max(slices[0], 0), min(slices[-1] + 1, A.shape[2])
        r0, r1 = max(rows[0] - border, 0), min(rows[-1] + border + 1, A.shape[0])
        c0, c1 = max(cols[0] - border, 0), min(cols[-1] + border + 1, A.shape[1])
        return (A[r0:r1, c0:c1, s0:s1], list(range(r0, r1)), list(range(c0, c1)),
                list(range(s0, s1)))

    def pickleMe(self, pickle_path='C:/PIRL/data/VentPickle.pkl'):
        """Vent_Analysis.py:542-553: every picklable attribute into one dict."""
        d = {}
        for attr in vars(self):
            try:
                pickle.dumps(getattr(self, attr))
                d[attr] = getattr(self, attr)
            except (pickle.PicklingError, AttributeError, TypeError):
                print(f"\033[31mSkipping non-picklable attribute: {attr}\033[37m")
        with open(pickle_path, 'wb') as f:
            pickle.dump(d, f)
        print(f'\033[32mPickled dictionary saved to {pickle_path}\033[37m')

    def unPickleMe(self, pickle_dict):
        for attr, value in pickle_dict.items():
            setattr(self, attr, value)

    def exportNifti(self, filepath=None, fileName=None):
        """Vent_Analysis.py:273-290: build4DdataArray() as <fileName>_dataArray.nii (NIfTI-1,
        identity affine; vent_analysis_amd.nifti, no nibabel needed).  The reference opens a
        folder dialog when filepath is None; here filepath is required."""
        print('\033[34mexportNifti method called...\033[37m')
        if filepath is None:
            raise ValueError("exportNifti: filepath is required (the reference asks with a "
                             "folder dialog)")
        if fileName is None:
            fileName = str(self.metadata['PatientName']).replace('^', '_')
        try:
            dataArray = self.build4DdataArray()
            savepath = os.path.join(filepath, fileName + '_dataArray.nii')
            nifti.save(savepath, dataArray, affine=np.eye(4))
            print(f'\033[32mNifti HPvent array saved to {savepath}\033[37m')
        except Exception:
            print('\033[31mCould not Export 4D HPvent mask Nifti...\033[37m')

    def exportDICOM(self, ds, save_dir='C:/PIRL/data/', optional_text='', forPACS=True):
        """Vent_Analysis.py:381-428.  The RGB defect overlay is rendered on the GPU (vh_overlay,
        csrc/export.hip) and returned as uint8 [slices][rows][cols][3]; with a dataset ``ds``
        (vent_analysis_amd.dicom.Dataset, or any object with pydicom-style attributes and
        save_as) the reference's files are written: one multi-frame RGB object (forPACS=False,
        :393-404) or one file per slice under save_dir/defectDICOMS (:405-428)."""
        if self.metadata['VDP'] == '':
            print('\033[31mCant export dicoms until you run calculate_VDP()...\033[37m')
            return None
        rgb = _lib.overlay(np.asarray(self.N4HPvent), np.asarray(self.defectArray),
                           device=self.device)
        if ds is None:
            return rgb
        from .dicom import generate_uid
        desc = f"{optional_text} - VDP: {np.round(self.metadata['VDP'], 1)}"
        R, C, Z = np.shape(self.N4HPvent)
        if forPACS is False:
            ds.PhotometricInterpretation = 'RGB'
            ds.SamplesPerPixel = 3
            ds.Rows, ds.Columns, ds.NumberOfFrames = R, C, Z
            ds.BitsAllocated = ds.BitsStored = 8
            ds.HighBit = 7
            ds.SOPInstanceUID = ds.SeriesInstanceUID = generate_uid()
            ds.PixelData = rgb.tobytes()
            ds.SeriesDescription = desc
            save_path = os.path.join(save_dir, f"{self.metadata['PatientName']}_defectDICOM.dcm")
            ds.save_as(save_path)
            print(f'\033[32mdefect DICOM saved to {save_path}\033[37m')
        else:
            try:   # the reference re-keys the study's own header (:406-407)
                self.ds.SeriesInstanceUID = generate_uid()
            except AttributeError:   # array-constructed object: self.ds is ''
                pass
            dicom_path = os.path.join(save_dir, 'defectDICOMS')
            os.makedirs(dicom_path, exist_ok=True)
            for i in range(Z):
                ds.BitsAllocated = 8
                ds.PixelData = rgb[i].tobytes()
                ds.Rows, ds.Columns = R, C
                ds.SamplesPerPixel = 3
                ds.PhotometricInterpretation = 'RGB'
                ds.BitsStored = 8
                ds.SeriesDescription = desc
                ds.InstanceNumber = i + 1
                ds.SliceLocation = i
                ds.SOPInstanceUID = generate_uid()
                ds.NumberOfFrames = 1
                ds.save_as(os.path.join(dicom_path, f"dicom_{i}.dcm"))
        return rgb

    def screenShot(self, path='C:/PIRL/data/screenShotTest.png', normalize95=False, parula=None):
        """Vent_Analysis.py:458-520: the 7-row montage (blank, blank, proton, HPvent, N4 + mask
        border, N4 + defects, N4 + parula CI) over cropToData(mask, border=5), rendered on the
        GPU (vh_montage) as the uint8(IMAGE * 255) array, returned and -- when PIL is present --
        saved as PNG with the reference's text annotations (:500-518: slice numbers, patient,
        disease, dates, volumes, DE / FEV1 / VDP / CI, version, user and date; same positions,
        strings and sizes).  The reference draws them in arial.ttf; where that font is missing
        PIL's default font at the same size stands in (text pixels then differ: parity unpinned).
        parula: the 64 x 3 colour table the reference loads from 'C:\\PIRL\\data\\parula.np.npy'
        (same default path).  The returned array is the montage without the text."""
        if parula is None:
            parula = np.load('C:\\PIRL\\data\\parula.np.npy', allow_pickle=False)
        _, rr, cc, ss = self.cropToData(self.mask, border=5)
        crop = (rr[0], len(rr), cc[0], len(cc), ss[0], len(ss))
        ci = None if isinstance(self.CIarray, str) else np.asarray(self.CIarray)
        proton = self.proton if not isinstance(self.proton, str) else np.zeros_like(self.HPvent)
        img = _lib.montage(np.asarray(proton), np.asarray(self.HPvent), np.asarray(self.N4HPvent),
                           np.asarray(self.mask_border), np.asarray(self.defectArray), ci,
                           np.asarray(parula), crop, device=self.device)
        try:
            from PIL import Image
        except ImportError:
            return img
        if path:
            image = Image.fromarray(img)
            self._annotate_screenshot(image, len(rr), len(cc), ss, img.shape[1])
            image.save(path, 'PNG')
            print(f'\033[32mScreenshot saved to {path}\033[37m')
        return img

    def _annotate_screenshot(self, image, h0, w0, ss, width):
        """The text of Vent_Analysis.py:500-518 on the montage; h0, w0 = the cropped volume's rows
        and columns (the reference's N4.shape[0], N4.shape[1]), width = the montage's width."""
        import datetime
        from PIL import ImageDraw, ImageFont

        def font(size):
            try:
                return ImageFont.truetype('arial.ttf', size=size)
            except OSError:   # the reference's font is not installed: PIL's default, same size
                try:
                    return ImageFont.load_default(size=size)
                except TypeError:   # Pillow < 10.1 (the reference pins 10.0.0): no size argument
                    return ImageFont.load_default()

        md, white = self.metadata, (255, 255, 255)
        draw = ImageDraw.Draw(image)
        for k in ss:
            draw.text((k * w0 - w0 / 2, h0 * 1.8), f"{k + 1}", fill=white, font=font(30))
        draw.text((10, h0 * 0.10), f"Patient: {md['PatientName']} ({md['PatientAge']}/{md['PatientSex']})",
                  fill=white, font=font(40))
        draw.text((10, h0 * 0.40), f"Disease: {md['Disease']}", fill=white, font=font(35))
        draw.text((10, h0 * 0.70), f"StudyDate: {md['StudyDate']}", fill=white, font=font(35))
        draw.text((10, h0 * 1.00), f"Visit#: {md['visit']}", fill=white, font=font(35))
        draw.text((10, h0 * 1.30), f"Treatment: {md['treatment']}", fill=white, font=font(35))
        draw.text((np.round(width * .25), h0 * 0.10), f"Lung Volume: {np.round(md['LungVolume'] * 1000)} mL",
                  fill=white, font=font(35))
        draw.text((np.round(width * .25), h0 * 0.40), f"Defect Volume: {np.round(md['DefectVolume'] * 1000)} mL",
                  fill=white, font=font(35))
        draw.text((np.round(width * .50), h0 * 0.10), f"DE: {md['DE']} mL", fill=white, font=font(35))
        draw.text((np.round(width * .50), h0 * 0.40), f"FEV1: {md['FEV1']} %", fill=white, font=font(35))
        draw.text((np.round(width * .50), h0 * 0.70), f"VDP: {np.round(md['VDP'], 1)} %", fill=white, font=font(35))
        try:   # as the reference: no CI line when the CI is not numeric yet
            draw.text((np.round(width * .50), h0 * 1.00), f"CI: {np.round(md['CI'])} %", fill=white, font=font(35))
        except Exception:
            pass
        draw.text((np.round(width * .75), h0 * 0.25), f'Analysis Version: {self.version}', fill=white, font=font(35))
        draw.text((np.round(width * .75), h0 * 0.50),
                  f"Analyzed by: {md['analysisUser']} on {str(datetime.datetime.today()).split()[0]}",
                  fill=white, font=font(35))

    def process_RAW(self, filepath=None, raw_K=None):
        """TWIX reconstruction (Vent_Analysis.py:522-540): raw_HPvent = transpose(fftshift(fft2(
        fftshift(raw_K[:, :, k]))), (1, 0, 2))[:, ::-1, :] in complex128, on the GPU (vh_recon).
        The twix parse (mapvbvd.mapVBVD, :532-536) needs mapvbvd, which is not installed here: pass
        the squeezed k-space array as raw_K instead (what ``twix.image['']`` returns)."""
        if raw_K is None:
            try:
                import mapvbvd  # noqa: F401  (not in the reference's requirements either)
            except ImportError as e:
                raise ImportError("process_RAW: reading a twix file needs mapvbvd; pass raw_K= "
                                  "(the squeezed k-space array) instead") from e
            twix = mapvbvd.mapVBVD(filepath)
            self.raw_twix = twix
            self.metadata['TWIXscanDateTime'] = twix.hdr.Config['PrepareTimestamp']
            self.metadata['TWIXprotocolName'] = twix.hdr.Meas['tProtocolName']
            twix.image.squeeze = True
            raw_K = twix.image['']
        self.raw_K = np.asarray(raw_K)
        self.raw_HPvent = _lib.recon(self.raw_K)

    def __repr__(self):
        s = f'\033[35mVent_Analysis\033[37m class object version \033[94m{self.version}\033[37m\n'
        for attr, value in vars(self).items():
            if isinstance(value, np.ndarray):
                s += f'\033[32m {attr}: \033[36m{value.shape} \033[37m\n'
            elif isinstance(value, dict):
                for a2, v2 in value.items():
                    s += f'   \033[32m {a2}: \033[36m{v2} \033[37m\n'
            elif isinstance(value, str) and value == '':
                s += f'\033[31m {attr}: \033[37m\n'
            else:
                s += f'\033[32m {attr}: \033[36m{type(value)} \033[37m\n'
        return s
