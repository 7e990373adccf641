import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libventhip.so)")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "vdp_*.npz")))


def load_case(path):
    """Inputs + expected outputs of one golden case (inputs regenerated from the seed and checked
    against the stored sha256, or stored verbatim for the edge case)."""
    from vent_analysis_amd.synth import synth_volume, volume_digest
    g = dict(np.load(path))
    shape = tuple(int(s) for s in g["shape"])
    if "hp" in g:
        X, M = g["hp"], g["mask"].astype(np.float64)
    else:
        X, M = synth_volume(*shape, int(g["seed"]))
        assert volume_digest(X, M) == g["input_sha256"].item().decode(), "synthetic input drift"
    n = int(np.prod(shape))
    unp = lambda k: np.unpackbits(g[k])[:n].reshape(shape)  # noqa: E731
    exp = dict(defect=unp("defect"), defect_border=unp("defect_border").astype(bool),
               mask_border=unp("mask_border"), lb=g["lb"])
    for k in ("SNR", "VDP", "VDP_lb", "LungVolume", "DefectVolume", "mean_anchor", "p99",
              "CI", "ci_values"):
        if k in g:
            exp[k] = g[k]
    return X, M, g["vox"], exp, os.path.basename(path)


@pytest.fixture(scope="session")
def cases():
    return [load_case(p) for p in golden_files()]
