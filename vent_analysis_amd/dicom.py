"""Minimal DICOM Part-10 reader/writer for the ingest row.

The reference reads studies with ``pydicom.dcmread`` (Vent_Analysis.py:169-196) and pulls the
header elements of Vent_Analysis.py:198-223.  pydicom is not installed in this image, so this
module restates the part of the DICOM standard (PS3.5 / PS3.10) those call sites use:

* the 128-byte preamble + ``DICM`` + File Meta group (explicit VR little endian);
* data sets in Implicit VR Little Endian (1.2.840.10008.1.2), Explicit VR Little Endian
  (1.2.840.10008.1.2.1) or Explicit VR Big Endian (1.2.840.10008.1.2.2);
* nested sequences with defined or undefined lengths (the per-frame functional groups
  ``ds[0x5200, 0x9230][k]['PixelMeasuresSequence'][0].PixelSpacing`` of :210);
* ``pixel_array`` for native (uncompressed) pixel data: shape (frames, rows, cols) for multi-frame
  objects, (rows, cols) for single frames, dtype from BitsAllocated / PixelRepresentation like
  pydicom's numpy handler (no modality LUT / rescale applied).  Encapsulated (compressed) pixel
  data raises NotImplementedError.

Access mirrors the pydicom idioms of the reference: ``ds['PatientName'].value``, ``ds.Rows``,
``ds[0x5200, 0x9230][k]``, ``item['PixelMeasuresSequence'][0].PixelSpacing``.  ``write_dataset``
emits Explicit VR Little Endian files (test fixtures and exports).

Parity: pydicom is absent, so there is no reference output to pin against; the reader is checked
against files written from the standard's encoding rules (tests/test_dicom.py) -- parity unpinned.
"""
from __future__ import annotations

import os
import struct

import numpy as np

__all__ = ["Dataset", "DataElement", "dcmread", "write_dataset", "InvalidDicomError", "tag_for"]

IMPLICIT_LE = "1.2.840.10008.1.2"
EXPLICIT_LE = "1.2.840.10008.1.2.1"
EXPLICIT_BE = "1.2.840.10008.1.2.2"

# keyword -> (tag, VR) for the elements the reference's ingest reads, the pixel module, and the
# sequences of the enhanced multi-frame functional groups (implicit VR needs the VR from here)
_DICT = {
    "FileMetaInformationGroupLength": (0x00020000, "UL"),
    "FileMetaInformationVersion": (0x00020001, "OB"),
    "MediaStorageSOPClassUID": (0x00020002, "UI"),
    "MediaStorageSOPInstanceUID": (0x00020003, "UI"),
    "TransferSyntaxUID": (0x00020010, "UI"),
    "ImplementationClassUID": (0x00020012, "UI"),
    "SOPClassUID": (0x00080016, "UI"),
    "SOPInstanceUID": (0x00080018, "UI"),
    "StudyDate": (0x00080020, "DA"),
    "SeriesDate": (0x00080021, "DA"),
    "StudyTime": (0x00080030, "TM"),
    "SeriesTime": (0x00080031, "TM"),
    "Modality": (0x00080060, "CS"),
    "SeriesDescription": (0x0008103E, "LO"),
    "SliceLocation": (0x00201041, "DS"),
    "PatientName": (0x00100010, "PN"),
    "PatientID": (0x00100020, "LO"),
    "PatientBirthDate": (0x00100030, "DA"),
    "PatientSex": (0x00100040, "CS"),
    "PatientAge": (0x00101010, "AS"),
    "PatientSize": (0x00101020, "DS"),
    "PatientWeight": (0x00101030, "DS"),
    "SliceThickness": (0x00180050, "DS"),
    "SpacingBetweenSlices": (0x00180088, "DS"),
    "StudyInstanceUID": (0x0020000D, "UI"),
    "SeriesInstanceUID": (0x0020000E, "UI"),
    "InstanceNumber": (0x00200013, "IS"),
    "ImagePositionPatient": (0x00200032, "DS"),
    "ImageOrientationPatient": (0x00200037, "DS"),
    "PlanePositionSequence": (0x00209113, "SQ"),
    "PlaneOrientationSequence": (0x00209116, "SQ"),
    "FrameContentSequence": (0x00209111, "SQ"),
    "SamplesPerPixel": (0x00280002, "US"),
    "PhotometricInterpretation": (0x00280004, "CS"),
    "PlanarConfiguration": (0x00280006, "US"),
    "NumberOfFrames": (0x00280008, "IS"),
    "Rows": (0x00280010, "US"),
    "Columns": (0x00280011, "US"),
    "PixelSpacing": (0x00280030, "DS"),
    "BitsAllocated": (0x00280100, "US"),
    "BitsStored": (0x00280101, "US"),
    "HighBit": (0x00280102, "US"),
    "PixelRepresentation": (0x00280103, "US"),
    "RescaleIntercept": (0x00281052, "DS"),
    "RescaleSlope": (0x00281053, "DS"),
    "PixelMeasuresSequence": (0x00289110, "SQ"),
    "SharedFunctionalGroupsSequence": (0x52009229, "SQ"),
    "PerFrameFunctionalGroupsSequence": (0x52009230, "SQ"),
    "PixelData": (0x7FE00010, "OW"),
}
_BY_TAG = {t: (kw, vr) for kw, (t, vr) in _DICT.items()}

_LONG_VR = {"OB", "OD", "OF", "OL", "OV", "OW", "SQ", "SV", "UC", "UN", "UR", "UT", "UV"}
_STR_VR = {"AE", "AS", "CS", "DA", "DS", "DT", "IS", "LO", "LT", "PN", "SH", "ST", "TM", "UC",
           "UI", "UR", "UT"}
_TEXT_VR = {"LT", "ST", "UT"}   # single-valued free text: backslash is not a separator
_NUM_VR = {"US": "H", "SS": "h", "UL": "I", "SL": "i", "FL": "f", "FD": "d", "UV": "Q", "SV": "q"}
_ITEM, _ITEM_END, _SEQ_END = 0xFFFEE000, 0xFFFEE00D, 0xFFFEE0DD
_UNDEFINED = 0xFFFFFFFF


def generate_uid():
    """A fresh UID under the 2.25 (UUID-derived) root, as pydicom.uid.generate_uid(None) makes."""
    import uuid
    return "2.25." + str(uuid.uuid4().int)


class InvalidDicomError(Exception):
    """Not a DICOM Part-10 file (no ``DICM`` marker) -- pydicom's error of the same name."""


def tag_for(key):
    """Tag (int) of a keyword, an int tag, or a (group, element) pair."""
    if isinstance(key, str):
        if key not in _DICT:
            raise KeyError(key)
        return _DICT[key][0]
    if isinstance(key, tuple):
        return (int(key[0]) << 16) | int(key[1])
    return int(key)


class DataElement:
    __slots__ = ("tag", "VR", "value", "keyword")

    def __init__(self, tag, VR, value):
        self.tag = tag
        self.VR = VR
        self.value = value
        self.keyword = _BY_TAG.get(tag, ("", ""))[0]

    def __getitem__(self, k):   # a sequence element indexes its items (ds[0x5200, 0x9230][k])
        return self.value[k]

    def __len__(self):
        return len(self.value)

    def __repr__(self):
        return (f"({self.tag >> 16:04X},{self.tag & 0xFFFF:04X}) {self.keyword or '?'} "
                f"{self.VR}: {self.value!r}")


class Dataset:
    """Ordered tag -> DataElement map with pydicom-style keyword access."""

    def __init__(self):
        self._elems = {}
        self.file_meta = None
        self.is_little_endian = True
        self.is_implicit_VR = False

    def __contains__(self, key):
        try:
            return tag_for(key) in self._elems
        except KeyError:
            return False

    def __getitem__(self, key):
        return self._elems[tag_for(key)]

    def __setitem__(self, key, elem):
        self._elems[tag_for(key)] = elem

    def __getattr__(self, name):
        if name.startswith("_") or name not in _DICT:
            raise AttributeError(name)
        elems = self.__dict__.get("_elems", {})
        t = _DICT[name][0]
        if t not in elems:
            raise AttributeError(name)
        return elems[t].value

    def __setattr__(self, name, value):
        """pydicom-style ds.Keyword = value for the keywords this module knows (exportDICOM,
        Vent_Analysis.py:394-421); other names are plain attributes."""
        if name in _DICT:
            t, vr = _DICT[name]
            if name == "PixelData" and isinstance(value, (bytes, bytearray)):
                bits = self.get("BitsAllocated", 16)
                vr = "OB" if bits == 8 else "OW"
            self._elems[t] = DataElement(t, vr, value)
        else:
            object.__setattr__(self, name, value)

    def save_as(self, path):
        """pydicom's Dataset.save_as (Explicit VR Little Endian Part-10 file)."""
        write_dataset(path, self)

    def __iter__(self):
        return iter(self._elems[t] for t in sorted(self._elems))

    def __len__(self):
        return len(self._elems)

    def add_new(self, key, VR, value):
        t = tag_for(key)
        self._elems[t] = DataElement(t, VR, value)

    def get(self, key, default=None):
        try:
            return self[key].value
        except KeyError:
            return default

    @property
    def pixel_array(self):
        return _pixel_array(self)


# ---- decoding ------------------------------------------------------------------------------
def _decode_value(vr, raw, little):
    if vr in _STR_VR:
        s = raw.decode("latin-1").rstrip("\x00 ")
        parts = [s] if vr in _TEXT_VR else s.split("\\")
        if vr == "DS":
            vals = [float(p) for p in parts if p.strip() != ""]
        elif vr == "IS":
            vals = [int(float(p)) for p in parts if p.strip() != ""]
        elif vr in _TEXT_VR or vr == "PN":
            vals = [p.rstrip(" ") for p in parts]
        else:
            vals = [p.strip(" ") for p in parts]
        if not vals:
            return None if vr in ("DS", "IS") else ""
        return vals[0] if len(vals) == 1 else vals
    if vr in _NUM_VR:
        fmt = _NUM_VR[vr]
        size = struct.calcsize(fmt)
        n = len(raw) // size
        if n == 0:
            return None
        vals = list(struct.unpack(("<" if little else ">") + fmt * n, raw[:n * size]))
        return vals[0] if n == 1 else vals
    if vr == "AT":
        n = len(raw) // 4
        hw = struct.unpack(("<" if little else ">") + "H" * (2 * n), raw[:4 * n])
        vals = [(hw[2 * i] << 16) | hw[2 * i + 1] for i in range(n)]
        return vals[0] if n == 1 else vals
    return bytes(raw)   # OB / OW / OF / OD / OL / UN: raw bytes (byte order of the file)


class _Reader:
    def __init__(self, buf, little, implicit):
        self.buf = buf
        self.little = little
        self.implicit = implicit
        self.u16 = struct.Struct("<H" if little else ">H")
        self.u32 = struct.Struct("<I" if little else ">I")

    def _tag(self, pos):
        if pos + 4 > len(self.buf):
            raise ValueError("truncated element header")
        g = self.u16.unpack_from(self.buf, pos)[0]
        e = self.u16.unpack_from(self.buf, pos + 2)[0]
        return (g << 16) | e

    def header(self, pos):
        """(tag, VR, length, value offset) of the element at pos."""
        tag = self._tag(pos)
        if tag in (_ITEM, _ITEM_END, _SEQ_END):   # item markers: tag + 4-byte length, no VR
            return tag, None, self.u32.unpack_from(self.buf, pos + 4)[0], pos + 8
        if self.implicit:
            vr = _BY_TAG.get(tag, ("", "UN"))[1]
            length = self.u32.unpack_from(self.buf, pos + 4)[0]
            if vr == "UN" and length == _UNDEFINED:
                vr = "SQ"   # undefined length in implicit VR: a sequence (PS3.5 7.5)
            return tag, vr, length, pos + 8
        vr = self.buf[pos + 4:pos + 6].decode("ascii")
        if vr in _LONG_VR:
            return tag, vr, self.u32.unpack_from(self.buf, pos + 8)[0], pos + 12
        return tag, vr, self.u16.unpack_from(self.buf, pos + 6)[0], pos + 8

    def dataset(self, pos, end, in_item=False):
        """Elements from pos up to end, or up to the item delimiter when in_item."""
        ds = Dataset()
        ds.is_little_endian, ds.is_implicit_VR = self.little, self.implicit
        while pos < end:
            tag, vr, length, vpos = self.header(pos)
            if tag == _ITEM_END:
                if in_item:
                    return ds, vpos
                raise ValueError("item delimiter outside an item")
            if vr == "SQ" or (vr == "UN" and length == _UNDEFINED):
                items, pos = self.sequence(vpos, length)
                ds._elems[tag] = DataElement(tag, "SQ", items)
                continue
            if length == _UNDEFINED:   # encapsulated pixel data: keep the fragments
                frags, pos = self.fragments(vpos)
                ds._elems[tag] = DataElement(tag, vr, frags)
                continue
            raw = self.buf[vpos:vpos + length]
            if len(raw) != length:
                raise ValueError(f"element ({tag >> 16:04X},{tag & 0xFFFF:04X}) runs past the end")
            value = raw if tag == 0x7FE00010 else _decode_value(vr, raw, self.little)
            ds._elems[tag] = DataElement(tag, vr, value)
            pos = vpos + length
        if in_item:
            raise ValueError("item without a delimiter")
        return ds, pos

    def sequence(self, pos, length):
        items = []
        end = len(self.buf) if length == _UNDEFINED else pos + length
        while pos < end:
            tag, _, ilen, vpos = self.header(pos)
            if tag == _SEQ_END:
                return items, vpos
            if tag != _ITEM:
                raise ValueError(f"expected a sequence item, found ({tag >> 16:04X},{tag & 0xFFFF:04X})")
            if ilen == _UNDEFINED:
                item, pos = self.dataset(vpos, len(self.buf), in_item=True)
            else:
                item, _ = self.dataset(vpos, vpos + ilen)
                pos = vpos + ilen
            items.append(item)
        if length == _UNDEFINED:
            raise ValueError("sequence without a delimiter")
        return items, pos

    def fragments(self, pos):
        frags = []
        while True:
            tag, _, flen, vpos = self.header(pos)
            if tag == _SEQ_END:
                return ("encapsulated", frags), vpos
            if tag != _ITEM:
                raise ValueError("bad encapsulated pixel data")
            frags.append(bytes(self.buf[vpos:vpos + flen]))
            pos = vpos + flen


def dcmread(fp, force=False):
    """Read a DICOM file (path or binary file object) like ``pydicom.dcmread`` for the native
    transfer syntaxes above.  ``force=True`` accepts a file without the preamble/``DICM`` marker
    and reads it as Implicit VR Little Endian (pydicom's fallback)."""
    if hasattr(fp, "read"):
        buf = fp.read()
    else:
        with open(os.fspath(fp), "rb") as f:
            buf = f.read()
    buf = bytes(buf)
    meta = Dataset()
    if len(buf) >= 132 and buf[128:132] == b"DICM":
        r = _Reader(buf, little=True, implicit=False)
        tag, _, length, vpos = r.header(132)   # File Meta: explicit VR LE, led by its length
        if tag != 0x00020000:
            raise InvalidDicomError("File Meta group without its group length")
        glen = struct.unpack_from("<I", buf, vpos)[0]
        meta, pos = r.dataset(132, vpos + length + glen)
        ts = meta.get("TransferSyntaxUID", EXPLICIT_LE)
    elif force:
        pos, ts = 0, IMPLICIT_LE
    else:
        raise InvalidDicomError("File is missing the DICOM File Meta Information header (DICM); "
                                "use force=True to read it anyway")
    ts = str(ts).strip("\x00 ")
    if ts == IMPLICIT_LE:
        r = _Reader(buf, little=True, implicit=True)
    elif ts == EXPLICIT_BE:
        r = _Reader(buf, little=False, implicit=False)
    else:   # explicit VR little endian, and the encapsulated (compressed) syntaxes built on it
        r = _Reader(buf, little=True, implicit=False)
    ds, _ = r.dataset(pos, len(buf))
    ds.file_meta = meta
    ds.transfer_syntax = ts
    return ds


# ---- pixel data ----------------------------------------------------------------------------
def _pixel_array(ds):
    if 0x7FE00010 not in ds._elems:
        raise AttributeError("no PixelData element")
    raw = ds[0x7FE00010].value
    if isinstance(raw, tuple):
        raise NotImplementedError("encapsulated (compressed) pixel data is not supported; "
                                  "decompress the study to a native transfer syntax first")
    rows, cols = int(ds.Rows), int(ds.Columns)
    frames = int(ds.get("NumberOfFrames", 1) or 1)
    spp = int(ds.get("SamplesPerPixel", 1) or 1)
    bits = int(ds.BitsAllocated)
    signed = int(ds.get("PixelRepresentation", 0) or 0) == 1
    stored = int(ds.get("BitsStored", bits) or bits)
    if bits not in (8, 16, 32):
        raise NotImplementedError(f"BitsAllocated = {bits} is not supported")
    dt = np.dtype(("i" if signed else "u") + str(bits // 8))
    dt = dt.newbyteorder("<" if ds.is_little_endian else ">")
    n = rows * cols * frames * spp
    if len(raw) < n * dt.itemsize:
        raise ValueError(f"PixelData holds {len(raw)} bytes, {n * dt.itemsize} expected")
    arr = np.frombuffer(raw, dtype=dt, count=n).astype(dt.newbyteorder("="))
    if signed and stored < bits:   # sign-extend from BitsStored (pydicom's numpy handler)
        shift = bits - stored
        arr = (arr << shift) >> shift
    if spp == 1:
        return arr.reshape((frames, rows, cols) if frames > 1 else (rows, cols))
    if int(ds.get("PlanarConfiguration", 0) or 0) == 0:
        arr = arr.reshape(frames, rows, cols, spp)
    else:
        arr = arr.reshape(frames, spp, rows, cols).transpose(0, 2, 3, 1)
    return arr if frames > 1 else arr[0]


# ---- writing ---------------------------------------------------------------------------------
def _encode_value(vr, value, little=True):
    if vr in _STR_VR:
        vals = list(value) if isinstance(value, (list, tuple)) else [value]
        if vr == "DS":
            parts = [v if isinstance(v, str) else format(float(v), ".10g")[:16] for v in vals]
        elif vr == "IS":
            parts = [str(int(v)) for v in vals]
        else:
            parts = [str(v) for v in vals]
        b = "\\".join(parts).encode("latin-1")
        if len(b) % 2:
            b += b"\x00" if vr == "UI" else b" "
        return b
    if vr in _NUM_VR:
        vals = list(value) if isinstance(value, (list, tuple)) else [value]
        return struct.pack(("<" if little else ">") + _NUM_VR[vr] * len(vals), *vals)
    b = bytes(value)
    return b + b"\x00" if len(b) % 2 else b


class _Writer:
    def __init__(self, little=True, implicit=False, undefined_seq=False):
        self.little, self.implicit, self.undefined_seq = little, implicit, undefined_seq
        self.e = "<" if little else ">"

    def marker(self, tag, length):
        return struct.pack(self.e + "HHI", tag >> 16, tag & 0xFFFF, length)

    def head(self, tag, vr, length):
        if self.implicit:
            return struct.pack(self.e + "HHI", tag >> 16, tag & 0xFFFF, length)
        h = struct.pack(self.e + "HH", tag >> 16, tag & 0xFFFF) + vr.encode("ascii")
        if vr in _LONG_VR:
            return h + b"\x00\x00" + struct.pack(self.e + "I", length)
        return h + struct.pack(self.e + "H", length)

    def elements(self, out, ds):
        for elem in ds:
            tag, vr = elem.tag, elem.VR
            if vr == "SQ":
                body = bytearray()
                for item in elem.value:
                    ib = bytearray()
                    self.elements(ib, item)
                    if self.undefined_seq:
                        body += self.marker(_ITEM, _UNDEFINED) + ib + self.marker(_ITEM_END, 0)
                    else:
                        body += self.marker(_ITEM, len(ib)) + ib
                if self.undefined_seq:
                    out += self.head(tag, vr, _UNDEFINED) + body + self.marker(_SEQ_END, 0)
                else:
                    out += self.head(tag, vr, len(body)) + body
                continue
            val = _encode_value(vr, elem.value, self.little)
            out += self.head(tag, vr, len(val)) + val


def write_dataset(path, ds, undefined_length_sequences=False, transfer_syntax=EXPLICIT_LE):
    """Write ds as a Part-10 file (File Meta generated) in Explicit VR Little Endian, Implicit VR
    Little Endian or Explicit VR Big Endian.  Pixel data bytes are written as given, so they must
    already be in the target byte order."""
    if transfer_syntax not in (EXPLICIT_LE, IMPLICIT_LE, EXPLICIT_BE):
        raise ValueError(f"unsupported transfer syntax {transfer_syntax}")
    w = _Writer(little=transfer_syntax != EXPLICIT_BE, implicit=transfer_syntax == IMPLICIT_LE,
                undefined_seq=undefined_length_sequences)
    body = bytearray()
    w.elements(body, ds)
    meta = Dataset()
    meta.add_new("FileMetaInformationVersion", "OB", b"\x00\x01")
    meta.add_new("MediaStorageSOPClassUID", "UI", ds.get("SOPClassUID", "1.2.840.10008.5.1.4.1.1.4.1"))
    meta.add_new("MediaStorageSOPInstanceUID", "UI", ds.get("SOPInstanceUID", "1.2.3.4"))
    meta.add_new("TransferSyntaxUID", "UI", transfer_syntax)
    meta.add_new("ImplementationClassUID", "UI", "1.2.826.0.1.3680043.9.7433.1")
    mw = _Writer()
    mb = bytearray()
    mw.elements(mb, meta)
    gl = Dataset()
    gl.add_new("FileMetaInformationGroupLength", "UL", len(mb))
    glb = bytearray()
    mw.elements(glb, gl)
    with open(os.fspath(path), "wb") as f:
        f.write(b"\x00" * 128 + b"DICM" + bytes(glb) + bytes(mb) + bytes(body))
