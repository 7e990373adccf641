"""Debug: study vs sweep vs oracle after a fixed number of iterations (conv_threshold 0)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import native
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_volume

shape, seed = tuple(int(v) for v in sys.argv[1].split("x")), int(sys.argv[2])
X, M = synth_volume(*shape, seed)
for cm in (0, 1):
    for k in (1, 2, 3):
        kw = dict(max_iters=(k,), conv_threshold=0.0, conv_mode=cm)
        ref, its, conv = native.n4(X, M, **kw)
        outs = {}
        for drv in ("sweep", "study"):
            B = _lib.Batch(*shape, 1)
            B.upload(X[None], M.astype(np.uint8)[None])
            B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=drv, **kw))
            n4, *_, res = B.download(n4=True)
            B.close()
            outs[drv] = (n4[0], list(res[0].n4_iters[:1]), list(res[0].n4_conv[:1]))
        for drv, (o, i, c) in outs.items():
            d = np.abs(o.astype(np.float64) - ref) / np.abs(ref)
            print(f"cm{cm} k{k} {drv}: iters {i} conv {c} vs {list(conv)} maxrel {d.max():.3e} nbad {(d > 1e-6).sum()}")
