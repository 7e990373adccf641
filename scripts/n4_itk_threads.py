"""Spec (oracle/n4_oracle.c mode 0, what libventhip.so computes) against ITK's float restatement at
several thread counts T (n4_oracle_itk: ITK's per-thread fit lattices, summed after the threads, as
itk::BSplineScatteredDataPointSetToImageFilter splits the points over its work units).  SimpleITK
runs with the machine's core count by default, so "ITK's answer" depends on T; this prints how far
the spec is from each T and how far the T are from each other.  CPU only (test infrastructure).

  python3 scripts/n4_itk_threads.py [--big]     (--big: the 512^3 config-5 study, ~1 h on 8 cores)"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from oracle import native  # noqa: E402
from vent_analysis_amd.synth import synth_volume  # noqa: E402

THREADS = (1, 8, 16, 64)
CASES = [((128, 128, 16), 0, False), ((128, 128, 16), 1, False), ((128, 128, 24), 0, False),
         ((128, 128, 24), 1, False), ((128, 128, 24), 2, False), ((128, 128, 24), 3, False),
         ((96, 112, 20), 5, False), ((12, 70, 9), 12, False), ((12, 70, 9), 13, False),
         ((256, 256, 24), 7, False)]
CASES += [((128, 128, 24), s, True) for s in range(8)]   # bench.py's studies (vary=True), seeds 0-7
if "--big" in sys.argv:
    CASES = [((512, 512, 512), 11, False)]


def rel(a, b):
    return float(np.max(np.abs(a.astype(np.float64) - b) / np.abs(b.astype(np.float64))))


print("| study | spec iters | " + " | ".join(f"ITK T={t} iters" for t in THREADS) + " | "
      + " | ".join(f"spec vs T={t}" for t in THREADS) + " | max over T pairs |")
print("|---" * (2 + 2 * len(THREADS) + 1) + "|")
for shape, seed, vary in CASES:
    X, M = synth_volume(*shape, seed, vary=vary)
    t0 = time.time()
    a, ia, _ = native.n4(X, M, conv_mode=0)
    runs = {t: native.n4_itk(X, M, threads=t) for t in THREADS}
    fmt = lambda its: str(list(map(int, its)))  # noqa: E731
    pair = max(rel(runs[s][0], runs[t][0]) for s in THREADS for t in THREADS if s < t)
    tag = f"{'x'.join(map(str, shape))} s{seed}" + (" vary" if vary else "")
    print(f"| {tag} | {fmt(ia)} | " + " | ".join(fmt(runs[t][1]) for t in THREADS) + " | "
          + " | ".join(f"{rel(a, runs[t][0]):.1e}" for t in THREADS) + f" | {pair:.1e} |", flush=True)
    print(f"<!-- {tag}: {time.time() - t0:.0f} s -->", flush=True)
