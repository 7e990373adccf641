"""Distance of the N4 build spec (oracle/n4_oracle.c mode 0, what libventhip.so computes) from a
restatement of ITK's own float (RealType) arithmetic (mode 1: one thread, and ITK's per-thread fit
lattices at 16 threads), with a stage ablation: ITK-float with everything but one stage taken from
the spec ("spec but S5 ITK" isolates what the spec's fit precision contributes, etc.).  Prints the
DESIGN.md §6 table.  CPU only (test infrastructure: it calls the oracle).

  python3 scripts/n4_itk_distance.py [--big]     (--big adds the 512^3 config-5 study: ~15 min)"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import native  # noqa: E402
from vent_analysis_amd.synth import synth_volume  # noqa: E402

CASES = [((128, 128, 16), 0, False), ((128, 128, 16), 1, False), ((128, 128, 24), 0, False),
         ((128, 128, 24), 1, False), ((128, 128, 24), 2, False), ((128, 128, 24), 3, False),
         ((96, 112, 20), 5, False), ((12, 70, 9), 13, False), ((256, 256, 24), 7, False)]
CASES += [((128, 128, 24), s, True) for s in range(8)]   # bench.py's studies (vary=True), seeds 0-7
if "--big" in sys.argv:
    CASES.append(((512, 512, 512), 11, False))
SPEC_ALL = (1 << 1) | (1 << 3) | (1 << 5) | (1 << 6) | (1 << 7) | (1 << 9)


def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b) / np.abs(b.astype(np.float64))))


print("| study | spec iters | ITK-float iters | spec vs ITK | ITK 16 vs 1 thread | spec but S5 (fit) ITK | "
      "spec but S6 (eval) ITK | exact CoV (conv 1) iters | conv 1 vs ITK |")
print("|---|---|---|---|---|---|---|---|---|")
for shape, seed, vary in CASES:
    X, M = synth_volume(*shape, seed, vary=vary)
    t0 = time.time()
    a, ia, _ = native.n4(X, M, conv_mode=0)
    k1, ik1, _ = native.n4_itk(X, M, threads=1)
    k16, _, _ = native.n4_itk(X, M, threads=16)
    s5, i5, _ = native.n4_itk(X, M, spec=SPEC_ALL & ~(1 << 5))
    s6, i6, _ = native.n4_itk(X, M, spec=SPEC_ALL & ~(1 << 6))
    e, ie, _ = native.n4(X, M, conv_mode=1)
    fmt = lambda its: str(list(map(int, its)))  # noqa: E731
    tag = f"{'x'.join(map(str, shape))} s{seed}" + (" vary" if vary else "")
    print(f"| {tag} | {fmt(ia)} | {fmt(ik1)} | {rel(a, k1):.1e} | {rel(k16, k1):.1e} | "
          f"{rel(s5, k1):.1e}{'' if list(i5) == list(ik1) else ' ' + fmt(i5)} | "
          f"{rel(s6, k1):.1e}{'' if list(i6) == list(ik1) else ' ' + fmt(i6)} | {fmt(ie)} | "
          f"{rel(e, k1):.1e} |", flush=True)
