#!/bin/bash
# A/B builds: variants/liblorb_<name>.so with lorb_ba.hip compiled with extra flags, the rest from
# the regular build.  Variants live outside the package directory (lorb_slam_amd/ holds one library).
# usage: tools/build_variant.sh NAME "-DFLAG=1 ..."
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R/lorb_slam_amd/csrc" || exit 1
make -s || exit 1
mkdir -p _build_v "$R/variants"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $2 -c lorb_ba.hip -o _build_v/lorb_ba_$1.o || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o "$R/variants/liblorb_$1.so" _build_v/lorb_ba_$1.o \
  $(ls _build/*.o | grep -v '/lorb_ba.o') -lamdhip64 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
