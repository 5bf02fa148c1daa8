#!/bin/bash
# Diagnostic build: liblorb_stamps.so with -DLORB_CHOL_STAMPS (s_memtime phase stamps in the Cholesky)
cd "$(dirname "$0")/../lorb_slam_amd/csrc" || exit 1
mkdir -p _build_st
for f in *.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DLORB_CHOL_STAMPS $EXTRA -c "$f" -o "_build_st/${f%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o ../liblorb_stamps.so _build_st/*.o \
  -lamdhip64 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
