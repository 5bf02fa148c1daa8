#!/bin/bash
# A/B of several builds: tools/gpu_abn.sh NAME... times lorb_slam_amd/liblorb_NAME.so with
# tools/time_ba.py (C3 / C4 / C4x8 solves + per-kernel Schur / Cholesky times), each in its own step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
for v in "$@"; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so tools/gpu_step.sh 200 $O/abn_$v.log python tools/time_ba.py || exit $?
done
