"""ORACLE -- test infrastructure only.  numpy restatement of the TWIX reconstruction of
Vent_Analysis.process_RAW (/root/reference/Vent_Analysis.py:537-540), the checker for vh_recon.

The reference (numpy 1.23.2, requirements.txt:3) computes np.fft.fft2 in double precision whatever
the input dtype; numpy >= 2.0 keeps complex64 input in single precision, so the input is cast to
complex128 first to reproduce the pinned behaviour.  mapvbvd (the file parse, :532-536) is absent,
so this starts from the squeezed raw k-space array.  Parity: numpy's FFT itself is the reference's
arithmetic; the GPU's mixed-radix FFT rounds differently, so the tests compare within 1e-12 of each
slice's largest magnitude."""
from __future__ import annotations

import numpy as np


def process_raw(raw_K):
    """raw_HPvent of Vent_Analysis.process_RAW for the k-space array raw_K (n0, n1, nz)."""
    K = np.asarray(raw_K).astype(np.complex128)
    out = np.zeros(K.shape, np.complex128)                      # :537
    for k in range(K.shape[2]):                                 # :538-539
        out[:, :, k] = np.fft.fftshift(np.fft.fft2(np.fft.fftshift(K[:, :, k])))
    return np.transpose(out, (1, 0, 2))[:, ::-1, :]             # :540
