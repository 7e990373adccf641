"""Host-side DICOM ingest throughput: writes N synthetic 128x128x24 studies
(multi-frame uint16 xenon file + 24-file mask folder) to a scratch directory, then times
ingest.load_batch -> contiguous (B, R, C, Z) float32 / uint8 arrays.  Prints one JSON line.

usage: python scripts/ingest_bench.py [--studies 64] [--workers 8] [--dir /tmp/ingest_bench]
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))

from vent_analysis_amd import ingest  # noqa: E402
from test_dicom import synth_study, write_mask_folder, write_xenon  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--studies", type=int, default=64)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--shape", type=int, nargs=3, default=(128, 128, 24))
    ap.add_argument("--dir", default="/tmp/ingest_bench")
    a = ap.parse_args()
    shutil.rmtree(a.dir, ignore_errors=True)
    studies = []
    for s in range(a.studies):
        vol, mk = synth_study(*a.shape, seed=s % 16)
        d = os.path.join(a.dir, f"s{s:04d}")
        os.makedirs(d)
        write_xenon(os.path.join(d, "xe.dcm"), vol, (1.5, 1.5, 10.0))
        write_mask_folder(os.path.join(d, "mask"), mk)
        studies.append((os.path.join(d, "xe.dcm"), os.path.join(d, "mask")))
    ingest.load_batch(studies[:2], workers=a.workers)   # warm
    t0 = time.perf_counter()
    hp, mk, _ = ingest.load_batch(studies, workers=a.workers)
    dt = time.perf_counter() - t0
    nbytes = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(a.dir) for f in fs)
    print(json.dumps({"metric": "DICOM ingest studies/s (file + mask folder -> contiguous arrays)",
                      "value": round(a.studies / dt, 1), "unit": "studies/s",
                      "MB_per_s": round(nbytes / dt / 1e6, 1), "studies": a.studies,
                      "shape": list(a.shape), "workers": a.workers, "seconds": round(dt, 3)}))
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
