"""Debug: batch pipeline scalars vs the oracle chain on the GPU's N4 output."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from oracle import vdp_oracle as O
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch
for nb, do_n4 in ((3, True), (3, False), (1, True)):
    hp, mk = synth_batch(128, 128, 24, nb, base_seed=10)
    B = _lib.Batch(128, 128, 24, nb); B.upload(hp, mk)
    B.run(B.options(do_n4=do_n4, vox=(1.5, 1.5, 10.0), do_cohort=True))
    n4, d, bo, lb, res = B.download(n4=True); B.close()
    for b in range(nb):
        v = n4[b] if do_n4 else hp[b]
        s = np.sort(v[mk[b] > 0]).astype(np.float32)
        m = np.float32(np.mean(s)); p99 = s[int(len(s) * 0.99)]
        print(nb, do_n4, b, "mean", res[b].mean_anchor, m, "p99", res[b].p99, p99, "nmask", res[b].n_mask, len(s), "defect eq", int(res[b].n_defect), flush=True)
