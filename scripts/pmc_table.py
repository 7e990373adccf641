"""Summarise raw rocprofv3 --pmc passes per kernel class: counter totals per launch.

  python scripts/pmc_table.py DIR [DIR ...]
"""
import collections
import csv
import re
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
nl = collections.defaultdict(lambda: collections.defaultdict(set))
meta = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        nl[k][r["Counter_Name"]].add(r["Dispatch_Id"])
        meta[k] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
for k in sorted(tot):
    print(f"== {k}  vgpr/agpr/sgpr/lds {meta[k]}")
    for c in sorted(tot[k]):
        n = len(nl[k][c])
        print(f"   {c:28s} {tot[k][c] / n:16.1f} per launch ({n} launches)")
