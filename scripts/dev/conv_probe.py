"""Convergence-measure probe: oracle vs GPU drivers at a level capped at a fixed iteration count
(is an iteration-count mismatch a threshold tie or a real divergence?)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from oracle import native
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch
shape, nb, seed = (130, 20, 3), 2, 13
if len(sys.argv) > 1:
    shape = tuple(int(v) for v in sys.argv[1].split(",")); nb = int(sys.argv[2]); seed = int(sys.argv[3])
hp, mk = synth_batch(*shape, nb, base_seed=seed)
for b in range(nb):
    _, its, conv = native.n4(hp[b], mk[b])
    print("vol", b, "oracle its", list(its), "conv", list(conv), flush=True)
    for lev in range(4):
        cap = [50, 50, 50, 50][:lev] + [int(its[lev])] + [1] * (3 - lev)
        cap[:lev] = [int(v) for v in its[:lev]]
        _, _, c_o = native.n4(hp[b], mk[b], max_iters=tuple(cap))
        line = f"  level {lev} cap {cap} oracle {c_o[lev]:.9g}"
        for mode in ("study", "sweep"):
            B = _lib.Batch(*shape, 1); B.upload(hp[b:b+1], mk[b:b+1])
            B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=mode, max_iters=tuple(cap)))
            r = B.download(n4=False, maps=False)[4][0]; B.close()
            line += f" {mode} {r.n4_conv[lev]:.9g} its {list(r.n4_iters[:4])}"
        print(line, flush=True)
