#!/bin/bash
# A/B of several builds: tools/gpu_abn.sh NAME... times variants/liblorb_NAME.so (tools/build_variant.sh;
# NAME "main" = the regular lorb_slam_amd/liblorb.so) with tools/time_ba.py (C3 / C4 / C4x8 solves +
# per-kernel Schur / Cholesky times), each in its own step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
for v in "$@"; do
  lib=$R/variants/liblorb_$v.so; [ "$v" = main ] && lib=$R/lorb_slam_amd/liblorb.so
  LORB_LIB_PATH=$lib tools/gpu_step.sh 200 $O/abn_$v.log python tools/time_ba.py || exit $?
done
