"""Per-study durations of k_n4_study on bench.py's exact batch: one workgroup
per study, so the slowest study bounds the launch.  Prints per distinct study: iterations, masked
voxels n, wall time (us, device wall clock via vh_batch_study_times), and the tail summary; writes
the table as JSON to argv[1] when given."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from vent_analysis_amd import _lib  # noqa: E402
from vent_analysis_amd.synth import synth_batch  # noqa: E402

nb = 256
hp, mk = synth_batch(128, 128, 24, nb, base_seed=bench.shard_seed(0), unique=bench.BENCH_UNIQUE, vary=True)
B = _lib.Batch(128, 128, 24, nb)
B.upload(hp, mk)
o = B.options(do_n4=True, vox=(1.5, 1.5, 10.0), do_cohort=True)
runs = []
for rep in range(3):
    B.run(o)
    res = B.download(n4=False, maps=False)[4]
    runs.append(B.study_times())
us = np.median(np.stack(runs), axis=0)
its = np.array([sum(r.n4_iters[:4]) for r in res])
vm = (mk.reshape(nb, -1) == 1).sum(1)
rows = []
for b in range(bench.BENCH_UNIQUE):
    sel = np.arange(b, nb, bench.BENCH_UNIQUE)
    rows.append({"study": b, "iters": int(its[b]), "n": int(vm[b]), "us_mean": float(us[sel].mean()),
                 "us_min": float(us[sel].min()), "us_max": float(us[sel].max()),
                 "us_per_iter_per_kvoxel": float(us[sel].mean() / its[b] / (vm[b] / 1000.0))})
summ = {"min_us": float(us.min()), "mean_us": float(us.mean()), "max_us": float(us.max()),
        "max_over_mean": float(us.max() / us.mean()),
        "corr_us_iters_x_n": float(np.corrcoef(us, its * vm)[0, 1])}
print(json.dumps(summ))
for r in sorted(rows, key=lambda r: -r["us_mean"])[:12]:
    print(r)
if len(sys.argv) > 1:
    json.dump({"summary": summ, "studies": rows}, open(sys.argv[1], "w"), indent=1)
B.close()
