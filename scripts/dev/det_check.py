"""Study-driver determinism / oracle check on small batches (VH_LIB_PATH selects a variant)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
from oracle import native
from vent_analysis_amd import _lib
from vent_analysis_amd.synth import synth_batch
bad = 0
for shape, nb, seed in [((64, 64, 16), 3, 7), ((128, 128, 24), 4, 0), ((64, 64, 32), 3, 6)]:
    hp, mk = synth_batch(*shape, nb, base_seed=seed)
    its_ref = [list(native.n4(hp[b], mk[b])[1]) for b in range(nb)]
    for rep in range(3):
        B = _lib.Batch(*shape, nb); B.upload(hp, mk)
        B.run(B.options(do_n4=True, vox=(1.5, 1.5, 10.0), n4_mode="study"))
        res = B.download(n4=False, maps=False)[4]; B.close()
        its = [list(r.n4_iters[:4]) for r in res]
        ok = its == its_ref
        bad += not ok
        print(os.path.basename(os.environ.get("VH_LIB_PATH", "main")), shape, rep, "OK" if ok else f"BAD {its} ref {its_ref}", flush=True)
print("bad", bad)
