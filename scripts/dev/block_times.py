"""Per-study durations of k_n4_study (ST_PROF build: conv_level[7] = block wall time in us)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch
hp, mk = synth_batch(128, 128, 24, 256, base_seed=0, unique=16)
B = _lib.Batch(128, 128, 24, 256)
B.upload(hp, mk)
for rep in range(2):
    B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode="study"))
    res = B.download(n4=False, maps=False)[4]
d = np.array([r.n4_conv[3] for r in res])
its = np.array([sum(r.n4_iters[:4]) for r in res])
vm = (mk.reshape(256, -1) == 1).sum(1)
print("block us min/mean/max %.0f %.0f %.0f" % (d.min(), d.mean(), d.max()))
for s in range(16):
    sel = np.arange(s, 256, 16)
    print("seed", s, "iters", its[s], "vm", vm[s], "us mean %.0f min %.0f max %.0f" % (d[sel].mean(), d[sel].min(), d[sel].max()))
