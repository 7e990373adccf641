"""Per-launch HBM-side traffic of each kernel class from rocprofv3 --pmc passes.

  [BENCH_ARGS="--shape 256 256 24 --batch 1 ..."] python scripts/pmc_summary.py OUT.json DIR [DIR ...]

DIR/pmc_counter_collection.csv files from separate FETCH_SIZE / WRITE_SIZE passes
(scripts/gpu_pmc.sh).  Both counters are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE reports half the bytes of wide coalesced reads, so traffic =
2 * FETCH_SIZE + WRITE_SIZE.  Kernel names map to the library's timer classes (bench.py keys).  The summary records the
library's sha256 and the workload (bench.workload_key of the BENCH_ARGS the passes ran with, the
default bench command line when unset): bench.py prices a line's traffic only from a summary of the
same library and workload.
"""
import collections
import csv
import json
import sys

# (kernel-name key, timer class): classes timed around one kernel launch each (the multi-kernel
# classes n4_contract / n4_den / n4_init are not priced from counters)
CLASSES = [("k_n4_fit_items<0>", "n4_fit"), ("k_n4_fit<0>", "n4_fit"), ("k_n4_eval", "n4_eval"),
           ("k_n4_hist", "n4_hist"), ("k_n4_final", "n4_final"), ("k_n4_study", "n4_study"),
           ("k_n4_pcg2", "n4_pcg"), ("k_n4_pcg(", "n4_pcg"), ("k_n4_pcw", "n4_pcw"),
           ("k_n4_emap", "n4_emap"), ("k_plane<", "classify"), ("k_tile<true", "classify"),
           ("k_gather", "gather"), ("k_snr(", "snr"), ("k_sort_vol", "sort"),
           ("k_mask_stats", "mask_stats"), ("k_kmeans_s", "kmeans"), ("k_kmeans(", "kmeans")]


def klass(name):
    for key, cls in CLASSES:
        if key in name:
            return cls
    return None


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
            c = klass(r["Kernel_Name"])
            if c is None:
                continue
            tot[c][r["Counter_Name"]] += float(r["Counter_Value"]) * 1024.0
            launches[c][r["Counter_Name"]].add(r["Dispatch_Id"])
    res = {}
    for c, v in tot.items():
        if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
            continue
        nf, nw = len(launches[c]["FETCH_SIZE"]), len(launches[c]["WRITE_SIZE"])
        fetch, write = v["FETCH_SIZE"] / nf, v["WRITE_SIZE"] / nw
        res[c] = {"traffic_bytes_per_launch": 2.0 * fetch + write,
                  "fetch_size_bytes": fetch, "write_size_bytes": write, "launches": nf}
    import hashlib
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.environ.get("VH_LIB_PATH") or os.path.join(here, "vent_analysis_amd", "libventhip.so")
    # the library the passes ran: bench.py uses this summary's traffic only for the same build
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None
    import shlex
    sys.path.insert(0, here)
    import bench
    bargs = os.environ.get("BENCH_ARGS", "")
    wl = bench.workload_key(bench.make_parser().parse_args(shlex.split(bargs)))
    json.dump({"note": "traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (gfx950 FETCH_SIZE halving)",
               "lib_sha256": sha, "workload": wl, "bench_args": bargs, "kernels": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
