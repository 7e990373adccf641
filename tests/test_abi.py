"""CPU: the C-ABI library loads, exports every symbol include/vent_hip.h declares, its structs match
the ctypes mirror byte for byte, and the product path fails loudly instead of falling back."""
import ctypes as ct
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO
from vent_analysis_amd import _lib

HEADER = os.path.join(REPO, "include", "vent_hip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(vh_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib._SIGS, f"{n} has no ctypes signature"


def test_abi_version_and_status_strings():
    L = _lib.lib()
    assert L.vh_abi_version() == 8 == _lib.ABI_VERSION
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "vent_hip.h")).read()
    assert "#define VH_ABI_VERSION %d" % _lib.ABI_VERSION in hdr   # shim, header and library agree
    assert L.vh_status_string(0) == b"ok"
    assert b"maximum radius" in L.vh_status_string(_lib.VH_ERR_MAXRADIUS)


def test_struct_layouts_match_header(tmp_path):
    c = tmp_path / "sz.c"
    c.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
                 'int main(){printf("%%zu %%zu %%zu %%zu %%zu\\n", sizeof(vh_vdp_result), '
                 'sizeof(vh_run_opts), sizeof(vh_n4_params), offsetof(vh_run_opts, vox), '
                 'offsetof(vh_vdp_result, n_mask));}\n' % HEADER)
    exe = tmp_path / "sz"
    subprocess.run(["gcc", str(c), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == [ct.sizeof(_lib.VdpResult), ct.sizeof(_lib.RunOpts), ct.sizeof(_lib.N4Params),
                   _lib.RunOpts.vox.offset, _lib.VdpResult.n_mask.offset]


def test_default_params_are_simpleitk_defaults():
    p = _lib.n4_params()
    assert p.n_levels == 4 and list(p.max_iters)[:4] == [50] * 4
    assert abs(p.conv_threshold - 0.001) < 1e-7 and list(p.ncp) == [4, 4, 4]
    assert p.n_bins == 200 and p.spline_order == 3
    assert abs(p.wiener_noise - 0.01) < 1e-7 and abs(p.fwhm - 0.15) < 1e-7
    assert p.conv_mode == 0   # ITK's float Welford convergence measure (reference semantics)


def test_missing_library_fails_loudly(monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libventhip.so")
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(ImportError):
        _lib.lib()


@pytest.mark.skipif(_lib.device_count() > 0, reason="CPU-only container check")
def test_no_gpu_means_error_not_fallback():
    from vent_analysis_amd import Vent_Analysis
    M = np.zeros((8, 8, 4))
    M[2:6, 2:6, 1:3] = 1
    with pytest.raises(_lib.VentHipError):
        Vent_Analysis(xenon_array=np.ones((8, 8, 4), np.float32), mask_array=M, vox=(1, 1, 1))


def test_host_batch_shaping():
    a = np.arange(24, dtype=np.float64).reshape(2, 3, 4)
    b = _lib.as_batch(a.transpose(1, 2, 0), np.float32)     # non-contiguous DICOM-like view
    assert b.shape == (1, 3, 4, 2) and b.flags.c_contiguous and b.dtype == np.float32
    with pytest.raises(ValueError):
        _lib.as_batch(np.zeros((2, 2)), np.float32)


def test_mask_must_be_binary():
    from vent_analysis_amd.Vent_Analysis import _binary_u8
    assert _binary_u8(np.array([0.0, 1.0, 1.0]), "m").dtype == np.uint8
    with pytest.raises(ValueError):
        _binary_u8(np.array([0, 255]), "m")
