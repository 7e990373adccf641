"""GPU-box: N4 run-to-run determinism probe.  Runs one synthetic study several times on one batch
and prints iterations, final conv per level and the max relative difference to run 0."""
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_volume

R, C, Z = (int(v) for v in sys.argv[1].split("x"))
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 11
cm = int(os.environ.get("CONV_MODE", "0"))
X, M = synth_volume(R, C, Z, seed)
B = _lib.Batch(R, C, Z, 1)
B.upload(X[None], M.astype(np.uint8)[None])
o = B.options(do_n4=True, vox=(1.0, 1.0, 1.0), conv_mode=cm)
base = None
for r in range(reps):
    B.run(o)
    n4, _, _, _, res = B.download(n4=True, maps=False)
    its = list(res[0].n4_iters)[:4]
    conv = [float(c) for c in list(res[0].n4_conv)[:4]]
    if base is None:
        base = n4[0].copy()
        d = 0.0
    else:
        d = float(np.max(np.abs(n4[0] - base) / np.maximum(np.abs(base), 1e-30)))
    print(f"{R}x{C}x{Z} rep {r}: iters {its} conv {conv} maxrel_vs_rep0 {d:.3g}", flush=True)
B.close()
