"""Distance of the N4 build spec (oracle/n4_oracle.c mode 0, what libventhip.so computes) from a
restatement of ITK's own float (RealType) arithmetic (mode 1, single thread and with ITK's
per-thread fit lattices), on the golden seeds and the bench shape.  Prints the DESIGN.md §6 table.
CPU only (test infrastructure: it calls the oracle)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import native  # noqa: E402
from vent_analysis_amd.synth import synth_volume  # noqa: E402

CASES = [((128, 128, 16), 0), ((128, 128, 16), 1), ((128, 128, 24), 0), ((128, 128, 24), 1),
         ((128, 128, 24), 2), ((128, 128, 24), 3), ((96, 112, 20), 5), ((12, 70, 9), 13),
         ((256, 256, 24), 7)]


def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b) / np.abs(b.astype(np.float64))))


print("| study | spec (conv 0) iters | ITK-float 1 thread iters | max rel | ITK 16 threads vs 1 | "
      "exact CoV (conv 1) iters | max rel vs ITK |")
print("|---|---|---|---|---|---|---|")
for shape, seed in CASES:
    X, M = synth_volume(*shape, seed)
    t0 = time.time()
    a, ia, _ = native.n4(X, M, conv_mode=0)
    e, ie, _ = native.n4(X, M, conv_mode=1)
    k1, ik1, _ = native.n4_itk(X, M, threads=1)
    k16, ik16, _ = native.n4_itk(X, M, threads=16)
    print(f"| {'x'.join(map(str, shape))} s{seed} | {list(map(int, ia))} | {list(map(int, ik1))} | "
          f"{rel(a, k1):.1e} | {rel(k16, k1):.1e} | {list(map(int, ie))} | {rel(e, k1):.1e} |",
          flush=True)
