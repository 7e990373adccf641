"""Placement of the study kernel's workgroups (VH_STUDY_TRACE CSV from vh_batch_study_times:
batch, study, t_start, t_end, HW_ID, XCC_ID, wall-clock kHz): how many studies shared a CU at
once, and how long a study took alone vs beside another one."""
import collections
import sys

rows = []
for line in open(sys.argv[1]):
    bp, i, t0, t1, hw, xcc, khz = line.strip().split(",")[:7]
    hw = int(hw)
    cu = (int(xcc) & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF)
    rows.append((bp, int(i), int(t0), int(t1), cu, int(khz)))
khz = rows[0][5]
by_cu = collections.defaultdict(list)
for r in rows:
    by_cu[r[4]].append(r)
print(f"{len(rows)} studies on {len(by_cu)} CUs; studies per CU:",
      dict(sorted(collections.Counter(len(v) for v in by_cu.values()).items())))
alone, shared = [], []
for cu, rs in by_cu.items():
    for r in rs:
        ov = 0
        for q in rs:
            if q is r:
                continue
            ov += max(0, min(r[3], q[3]) - max(r[2], q[2]))
        dur = r[3] - r[2]
        (shared if ov > 0.5 * dur else alone).append(dur * 1000.0 / khz)
for name, v in (("mostly alone", alone), ("mostly shared", shared)):
    if v:
        print(f"{name}: {len(v)} studies, mean {sum(v) / len(v):.0f} us")
t0 = min(r[2] for r in rows)
t1 = max(r[3] for r in rows)
print(f"span {(t1 - t0) * 1000.0 / khz:.0f} us")
