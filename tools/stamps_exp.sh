#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
for v in stamps; do
  echo "== $v" >> gpurun_out/stamps_exp.log
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so timeout -k 10 120 python tools/chol_stamps.py >> gpurun_out/stamps_exp.log 2>&1 || exit 1
done
