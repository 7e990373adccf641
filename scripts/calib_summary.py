"""Summary of scripts/gpu_calib.sh: per access form of scripts/microbench/fetch_calib.hip, the
FETCH_SIZE and WRITE_SIZE of its dispatch (KiB -> bytes) over the bytes of the 128-B lines it
touched and over the bytes it used.

  python scripts/calib_summary.py PREFIX OUT.json   (PREFIX_m<mode>_<COUNTER>/ from gpu_calib.sh)"""
import csv
import glob
import json
import re
import sys

FORMS = {0: "16-B loads, coalesced", 1: "4-B loads, coalesced", 2: "4-B loads, one per 128-B line",
         3: "4-B loads, lanes 32 B apart", 4: "16-B stores, coalesced", 5: "4-B stores, coalesced",
         6: "4-B stores, one per 128-B line"}


def main():
    pre, out = sys.argv[1], sys.argv[2]
    res = {}
    for m, form in FORMS.items():
        row = {"form": form}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            log = open(f"{pre}_m{m}_{c}.log").read()
            g = re.search(r"lines (\d+) line_bytes (\d+) useful_bytes (\d+)", log)
            row["line_bytes"], row["useful_bytes"] = int(g.group(2)), int(g.group(3))
            files = glob.glob(f"{pre}_m{m}_{c}/**/*counter_collection.csv", recursive=True)
            v = 0.0
            for f in files:
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] == c and re.match(r"(void )?(ld|st)(4|16)\b", r["Kernel_Name"]):
                        v += float(r["Counter_Value"]) * 1024.0
            row[c.lower() + "_bytes"] = v
        row["fetch_over_line_bytes"] = row["fetch_size_bytes"] / row["line_bytes"]
        row["write_over_line_bytes"] = row["write_size_bytes"] / row["line_bytes"]
        res[m] = row
        print(m, form, "FETCH/lines %.3f WRITE/lines %.3f" % (row["fetch_over_line_bytes"],
                                                               row["write_over_line_bytes"]))
    json.dump({"note": "FETCH_SIZE / WRITE_SIZE of one dispatch over the bytes of the 128-B lines it "
                       "touched (1 GiB array, each line once; scripts/microbench/fetch_calib.hip)",
               "modes": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
