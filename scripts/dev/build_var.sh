#!/bin/bash
# Build a variant of libventhip.so with extra -D flags into scratch_libs/NAME.so (A/B on the GPU box).
# usage: scripts/dev/build_var.sh NAME -DFOO=1 ...
set -e
cd "$(dirname "$0")/../.."
NAME=$1; shift
B=/tmp/vb_$NAME; rm -rf $B; mkdir -p $B scratch_libs
mkdir -p $B/pkg $B/include; cp -r vent_analysis_amd/csrc $B/pkg/csrc; cp include/vent_hip.h $B/include/
rm -rf $B/pkg/csrc/build
make -s -C $B/pkg/csrc -j8 OUT=$PWD/scratch_libs/$NAME.so \
  CXXFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function -I/opt/rocm/include $*"
