#!/bin/bash
# build_flags.sh NAME "EXTRA FLAGS" -- libventhip.so variant with extra compile flags (e.g.
# "-DPC_PROF", "-DST_PROF") into scratch_libs/NAME.so for A/B and profiling runs (VH_LIB_PATH).
set -e
cd "$(dirname "$0")/../../vent_analysis_amd/csrc"
NAME=$1; FLAGS=$2
OBJ=/tmp/bf_$NAME; rm -rf $OBJ; mkdir -p $OBJ ../../scratch_libs
pids=()
for f in api vdp n4 n4_study ci export recon; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-function \
      -I/opt/rocm/include $FLAGS -c -o $OBJ/$f.o $f.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build_flags: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
    -o ../../scratch_libs/$NAME.so $OBJ/*.o
echo built scratch_libs/$NAME.so
