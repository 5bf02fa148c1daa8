#!/bin/bash
# GPU box: tools/time_ba.py against each lorb_slam_amd/liblorb_<v>.so given as arguments
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so timeout -k 10 120 python tools/time_ba.py 2>&1 | grep -E "^C4 W 1|^C3" || exit 1
done
