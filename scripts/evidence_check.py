"""Cross-check of bench lines against the kernel-trace statistics of the same build.

  python scripts/evidence_check.py [--strict] BENCH.json KERNEL_STATS.csv [BENCH.json KERNEL_STATS.csv ...]

For each (line, rocprofv3 --kernel-trace --stats summary) pair: the line's value, its roofline
(dominant kernel class by time per step, isolated launch time, frac, traffic and its source) and the
rocprofv3 average duration of the same kernel, and the fraction recomputed from that average
(the two must agree within 2 %).  With --strict the exit status is 1
when any pair disagrees by more than 2 % or a line's traffic is below its algorithmic bytes."""
import csv
import json
import sys

# timer class -> kernel names rocprofv3 reports for it (the first one present is used)
NAMES = {"n4_study": ["k_n4_study", "k_n4_studyg"], "n4_pcg": ["k_n4_pcg2", "k_n4_pcg"], "n4_pcw": ["k_n4_pcw"],
         "n4_fit": ["void k_n4_fit_items<0>"], "n4_eval": ["k_n4_eval"], "n4_hist": ["k_n4_hist"],
         "sort": ["k_sort_vol"], "kmeans": ["k_kmeans_s", "k_kmeans"], "n4_final": ["k_n4_final"],
         "ci_walk": ["k_ci_walk"], "classify": ["void k_plane<0, true>", "void k_plane<1, true>"]}


def check(bench_path, stats_path):
    line = json.loads([ln for ln in open(bench_path) if ln.startswith("{")][-1])
    r = line.get("roofline") or {}
    print(f"== {bench_path}")
    print("value", line["value"], line["unit"], "ms/step", line["ms_per_step"],
          "h2h", line.get("host_to_host_vol_s"))
    print("roofline", r.get("kernel"), "launches/step", r.get("launches_per_step"), "iso us",
          r.get("avg_launch_us"), "frac", r.get("frac"), "traffic", r.get("traffic"),
          "traffic/alg", r.get("traffic_over_alg"), "|", r.get("traffic_note"), r.get("traffic_source"))
    print("non_n4_us_per_step", r.get("non_n4_us_per_step"))
    rows = {x["Name"].split("(")[0]: x for x in csv.DictReader(open(stats_path))}
    ok = True
    cands = NAMES.get(r.get("kernel"), [r.get("kernel")])
    k = next((c for c in cands if c in rows), None)
    if k and r.get("alg_bytes_per_launch"):
        avg = float(rows[k]["AverageNs"]) * 1e-9
        frac = r["alg_bytes_per_launch"] / avg / 1e9 / r["peak"]
        dev = (r.get("frac", 0) / frac - 1) * 100
        print(f"rocprof {k}: {avg * 1e3:.4f} ms average over {rows[k]['Calls']} calls -> frac "
              f"{frac:.4f}; bench frac {r.get('frac')} ({dev:+.1f} %)")
        ok = abs(dev) <= 2.0
    else:
        print(f"rocprof: no row for {cands} in {stats_path}")
        ok = False
    if r.get("traffic_over_alg") is not None and r["traffic_over_alg"] < 1.0:
        print("traffic below the algorithmic bytes: not evidence")
        ok = False
    for name in list(rows)[:10]:
        x = rows[name]
        print(f"  {name[:40]:40s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:10.1f} us {x['Percentage']}")
    return ok


def main():
    argv = sys.argv[1:]
    strict = "--strict" in argv
    argv = [a for a in argv if a != "--strict"]
    if len(argv) < 2 or len(argv) % 2:
        sys.exit(__doc__)
    ok = all([check(argv[i], argv[i + 1]) for i in range(0, len(argv), 2)])
    print("ALL WITHIN 2 %" if ok else "SOME LINE OUTSIDE 2 % (or traffic below algorithmic)")
    sys.exit(1 if strict and not ok else 0)


if __name__ == "__main__":
    main()
