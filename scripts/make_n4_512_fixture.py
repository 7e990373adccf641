"""Pins N4 at BASELINE config-5 scale: runs the C oracle (oracle/n4_oracle.c, spec mode,
conv_mode 0 = ITK's float Welford) once on the synthetic 512^3 seed-11 study and stores

  iters[4], conv[4]                       per-level iterations / final convergence
  sample_idx, sample_val                  N4HPvent at a fixed strided voxel sample (float32)
  sha256                                  of the full float32 N4HPvent (C order)

in tests/golden/n4_512_seed11.npz (read by tests/test_gpu_parity.py
test_config5_512_cubed_n4_morph3d).  Build container only: ~2 min single-threaded, ~5 GB."""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from oracle import native  # noqa: E402
from vent_analysis_amd.synth import synth_volume  # noqa: E402

STRIDE = 4099   # prime: the sample walks every row / slice phase


def main():
    native.build()
    X, M = synth_volume(512, 512, 512, 11)
    t = time.time()
    out, its, conv = native.n4(X, M.astype(np.uint8), conv_mode=0)
    dt = time.time() - t
    flat = out.reshape(-1)
    idx = np.arange(0, flat.size, STRIDE, dtype=np.int64)
    sha = hashlib.sha256(np.ascontiguousarray(out, dtype=np.float32).tobytes()).hexdigest()
    dst = os.path.join(HERE, "..", "tests", "golden", "n4_512_seed11.npz")
    np.savez_compressed(dst, iters=np.asarray(its, np.int32), conv=np.asarray(conv, np.float32),
                        sample_idx=idx, sample_val=flat[idx].astype(np.float32),
                        sha256=np.array(sha), stride=np.int64(STRIDE), seconds=np.float64(dt))
    print(f"iters {list(its)} conv {list(conv)} sha256 {sha} ({dt:.1f} s) -> {os.path.normpath(dst)}")


if __name__ == "__main__":
    main()
