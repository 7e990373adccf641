"""Debug: k_n4_study vs sweeps vs oracle at a fixed number of single-level iterations."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from oracle import native
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch

def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b) / np.maximum(np.abs(b), 1e-30)))

shape = tuple(int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (128, 128, 24)
seed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
hp, mk = synth_batch(*shape, 2, base_seed=seed)
cases = [dict(max_iters=m) for m in [(50,), (50, 50), (50, 50, 50), (50, 50, 50, 50)]]
cases += [dict(max_iters=(50, 50, 50, 50), conv_threshold=0.0)]
cases += [dict(max_iters=(n,), conv_threshold=0.0) for n in (10, 20, 30, 50)]
for kw in cases:
    mi = kw["max_iters"]
    out = {}
    for mode in ("study", "sweep"):
        B = _lib.Batch(*shape, 2)
        B.upload(hp, mk)
        B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=mode, **kw))
        out[mode] = B.download(n4=True)
        B.close()
    ref, its, _ = native.n4(hp[0], mk[0], **kw)
    print(kw, "study-vs-oracle %.3g" % rel(out["study"][0][0], ref),
          "sweep-vs-oracle %.3g" % rel(out["sweep"][0][0], ref),
          "study-vs-sweep %.3g" % rel(out["study"][0][0], out["sweep"][0][0]),
          "iters", list(out["study"][4][0].n4_iters[:len(mi)]), list(its), flush=True)
