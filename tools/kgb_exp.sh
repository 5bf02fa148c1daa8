#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
for v in liblorb liblorb_g128 liblorb_g64; do
  echo "== $v" >> gpurun_out/kgb.log
  LORB_LIB_PATH=$R/lorb_slam_amd/$v.so timeout -k 10 120 python tools/time_ba.py >> gpurun_out/kgb.log 2>&1 || exit 1
done
