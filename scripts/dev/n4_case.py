"""GPU-box: one synthetic study through both N4 drivers and the C oracle; prints iterations and
convergence values (diagnostics for driver/oracle mismatches)."""
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_volume
from oracle import native

R, C, Z = (int(v) for v in sys.argv[1].split("x"))
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 11
cm = int(sys.argv[3]) if len(sys.argv) > 3 else 0
X, M = synth_volume(R, C, Z, seed)
ref, its_ref, conv_ref = native.n4(X, M.astype(np.uint8), conv_mode=cm)[:3]
print("oracle", list(its_ref), [float(c) for c in conv_ref])
for mode in ("sweep", "study"):
    B = _lib.Batch(R, C, Z, 1)
    B.upload(X[None], M.astype(np.uint8)[None])
    try:
        B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=mode, conv_mode=cm))
    except ValueError as e:
        print(mode, "skipped:", e)
        continue
    n4, _, _, _, res = B.download(n4=True, maps=False)
    B.close()
    print(mode, list(res[0].n4_iters[:4]), [float(c) for c in res[0].n4_conv[:4]],
          "maxrel", float(np.max(np.abs(n4[0] - ref) / np.maximum(np.abs(ref), 1e-30))))
