"""Debug: study driver on a 64x64x16 batch with / without an empty-mask volume."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from oracle import native
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch

def run(hp, mk, mode, **kw):
    B = _lib.Batch(*hp.shape[1:], hp.shape[0]); B.upload(hp, mk)
    B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode=mode, **kw))
    out = B.download(n4=True); B.close(); return out

hp, mk = synth_batch(64, 64, 16, 3, base_seed=7)
for empty in (False, True):
    m2 = mk.copy()
    if empty: m2[1] = 0
    for mode in ("study", "sweep"):
        n4, d, _, _, res = run(hp, m2, mode)
        print("empty", empty, mode, [list(r.n4_iters[:4]) for r in res], [list(np.round(r.n4_conv[:4], 6)) for r in res], flush=True)
    for b in (0, 2):
        print(" oracle", b, list(native.n4(hp[b], m2[b])[1]))
# single iterations
for mi in ((1,), (2,), (3,)):
    for mode in ("study", "sweep"):
        n4, d, _, _, res = run(hp, mk, mode, max_iters=mi, conv_threshold=0.0)
        print(mi, mode, float(n4[0].sum()), float(n4[2].sum()), flush=True)
    ref = native.n4(hp[0], mk[0], max_iters=mi, conv_threshold=0.0)[0]
    print(mi, "oracle", float(ref.sum()))
