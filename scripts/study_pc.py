"""Per-study S7 cost from a VH_STUDY_TRACE CSV (vh_batch_study_times): wall time against the PC
rounds, the frozen-mu serial runs at stage 0's cap (closed / stopped at its block budget) and the
serial fallbacks of the exact rounds, summed over the study's N4 iterations.  N4State.pc_fallbacks
packs them as fallbacks + 1000 (closes + 100 stops)."""
import sys

import numpy as np

rows = [l.strip().split(",") for l in open(sys.argv[1])]
khz = int(rows[0][6])
t = np.array([(int(r[3]) - int(r[2])) * 1000.0 / khz for r in rows])   # us
rnd = np.array([int(r[7]) for r in rows])
x = np.array([int(r[8]) for r in rows])
its = np.array([int(r[9]) for r in rows])
fb, fr = x % 1000, x // 1000
closes, stops = fr % 100, fr // 100
print(f"{len(rows)} studies: time mean {t.mean():.0f} us, max {t.max():.0f}; PC rounds per iteration "
      f"mean {rnd.sum() / its.sum():.2f} over {int(its.sum())} iterations")
print(f"frozen serial at stage 0's cap: {int(closes.sum())} closed, {int(stops.sum())} stopped at the budget; "
      f"serial fallbacks {int(fb.sum())} in {int((fb > 0).sum())} studies")
for name, sel in (("a serial fallback", fb > 0), ("a frozen-serial close", closes > 0)):
    if sel.any() and (~sel).any():
        print(f"mean time with / without {name}: {t[sel].mean():.0f} / {t[~sel].mean():.0f} us")
print("correlation of time with rounds / iterations:", round(float(np.corrcoef(t, rnd)[0, 1]), 3),
      round(float(np.corrcoef(t, its)[0, 1]), 3))
o = np.argsort(-t)[:12]
print("slowest (us, iterations, rounds, fallbacks, closes, stops):",
      [(int(t[i]), int(its[i]), int(rnd[i]), int(fb[i]), int(closes[i]), int(stops[i])) for i in o])
