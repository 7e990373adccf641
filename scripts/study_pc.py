"""Per-study S7 cost from a VH_STUDY_TRACE CSV (vh_batch_study_times): wall time against the PC
rounds and serial fallbacks the study took over all its N4 iterations."""
import sys

import numpy as np

rows = [l.strip().split(",") for l in open(sys.argv[1])]
khz = int(rows[0][6])
t = np.array([(int(r[3]) - int(r[2])) * 1000.0 / khz for r in rows])   # us
rnd = np.array([int(r[7]) for r in rows])
fbx = np.array([int(r[8]) for r in rows])
fb, wfb = fbx % 1000, fbx // 1000   # serial fallbacks of the exact rounds, wave-serial stage-0 finishes
its = np.array([int(r[9]) for r in rows])
print(f"{len(rows)} studies: time mean {t.mean():.0f} us, max {t.max():.0f}; PC rounds per iteration "
      f"mean {rnd.sum() / its.sum():.2f}; studies with a serial fallback {int((fb > 0).sum())} "
      f"({int(fb.sum())} fallbacks over {int(its.sum())} iterations)")
print(f"stage-0 wave-serial finishes: {int(wfb.sum())} in {int((wfb > 0).sum())} studies")
if (wfb > 0).any():
    print(f"mean time with / without a wave-serial finish: {t[wfb > 0].mean():.0f} / {t[wfb == 0].mean():.0f} us")
if (fb > 0).any():
    print(f"mean time with / without a fallback: {t[fb > 0].mean():.0f} / {t[fb == 0].mean():.0f} us")
print("correlation of time with rounds / iterations:", round(float(np.corrcoef(t, rnd)[0, 1]), 3),
      round(float(np.corrcoef(t, its)[0, 1]), 3))
o = np.argsort(-t)[:12]
print("slowest: (us, iterations, rounds, fallbacks)",
      [(int(t[i]), int(its[i]), int(rnd[i]), int(fb[i]), int(wfb[i])) for i in o])
