"""CPU: PC pass 0's exp (vent_analysis_amd/csrc/expf_small.h, the same source the kernels include)
equals the spec's p = (float)exp((double)d) (Vent_Analysis.py:330-331 -> ITK's float step, DESIGN
§4.2.1) -- checked here under g++ against glibc's exp on a strided sweep of every float with
|x| <= 2^-5, a dense run near 0 and near the 2^-5 edge, and arguments past it (the full exp).
Every float of the range was checked once (scripts/dev/expf_small_check.cpp: 2 046 820 354
arguments, 0 mismatches, 305 midpoint fallbacks)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "vent_analysis_amd", "csrc")
CHECK = os.path.join(HERE, "..", "scripts", "dev", "expf_small_check.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_expf_small_equals_double_exp(tmp_path):
    exe = str(tmp_path / "chk")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, CHECK, "-o", exe],
                   check=True)
    for lo, hi, stride in (("0", "0.03125", "1021"),          # the whole range, strided
                           ("0", "1e-30", "1"),               # dense near 0 (denormals included)
                           ("0.0312", "0.03125", "1"),        # dense at the edge
                           ("0.03125", "20", "4093")):        # past the edge: the full exp
        r = subprocess.run([exe, lo, hi, stride], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout
        assert " bad 0 " in r.stdout, r.stdout
