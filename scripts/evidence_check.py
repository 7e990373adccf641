"""Cross-check of a bench line against the kernel-trace statistics of the same build.

  python scripts/evidence_check.py BENCH.json KERNEL_STATS.csv

Prints the line's value, its roofline (kernel, isolated launch time, frac, traffic and source) and
the rocprofv3 average duration of the same kernel, and the fraction recomputed from that average
(the two must agree within 2 %).  Exit status 0 either way: this is a report."""
import csv
import json
import sys

NAMES = {"n4_study": "k_n4_study", "n4_pcg": "k_n4_pcg", "n4_pcw": "k_n4_pcw", "sort": "k_sort_vol",
         "kmeans": "k_kmeans", "n4_final": "k_n4_final", "ci_walk": "k_ci_walk"}


def main():
    line = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
    r = line.get("roofline") or {}
    print("value", line["value"], line["unit"], "ms/step", line["ms_per_step"],
          "h2h", line.get("host_to_host_vol_s"))
    print("roofline", r.get("kernel"), "iso us", r.get("avg_launch_us"), "frac", r.get("frac"),
          "traffic", r.get("traffic"), r.get("traffic_note"), r.get("traffic_source"))
    print("non_n4_us_per_step", r.get("non_n4_us_per_step"))
    rows = {x["Name"].split("(")[0]: x for x in csv.DictReader(open(sys.argv[2]))}
    k = NAMES.get(r.get("kernel"), r.get("kernel"))
    if k in rows and r.get("alg_bytes_per_launch"):
        avg = float(rows[k]["AverageNs"]) * 1e-9
        frac = r["alg_bytes_per_launch"] / avg / 1e9 / r["peak"]
        print(f"rocprof {k}: {avg * 1e3:.3f} ms average over {rows[k]['Calls']} calls -> frac "
              f"{frac:.4f}; bench frac {r.get('frac')} ({(r.get('frac', 0) / frac - 1) * 100:+.1f} %)")
    for name in list(rows)[:10]:
        x = rows[name]
        print(f"  {name[:32]:32s} {x['Calls']:>5s} {float(x['AverageNs']) / 1e3:10.1f} us {x['Percentage']}")


if __name__ == "__main__":
    main()
