#!/bin/bash
# GPU-box (round 4): stage 0's round cap before the frozen serial (PC_AMAX0 16 / 24 / 40) and its
# block budget (PC_FRZ_RUN 96 / 192): one batch with the per-study trace, then two in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4y}
for v in base a16_r96 a24_r96 a24_r192; do
  if [ $v = base ]; then L=""; else L=$PWD/scratch_ab/$v.so; fi
  VH_LIB_PATH=$L VH_STUDY_TRACE=gpurun_out/${TAG}_${v}.csv timeout -k 10 300 python bench.py --steps 4 --warmup 1 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_${v}_b1.json 2> gpurun_out/${TAG}_${v}_b1.err
  rc=$?; echo "$v b1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  VH_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_${v}_b2.json 2> gpurun_out/${TAG}_${v}_b2.err
  rc=$?; echo "$v b2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "== $v"; python3 scripts/study_pc.py gpurun_out/${TAG}_${v}.csv | head -3
  python3 - $TAG $v <<'PY'
import json, sys
for s in ("b1", "b2"):
    d = json.loads([l for l in open(f"gpurun_out/{sys.argv[1]}_{sys.argv[2]}_{s}.json") if l.startswith("{")][-1])
    print(s, d["value"], d["ms_per_step"], d["n4_study_times"])
PY
done
