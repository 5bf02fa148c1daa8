#!/bin/bash
# GPU box: BA parity tests + timings against lorb_slam_amd/liblorb_<v>.so for each variant argument
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ba.py > gpurun_out/vt_$v.log 2>&1 || { tail -15 gpurun_out/vt_$v.log; exit 1; }
  tail -1 gpurun_out/vt_$v.log
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so timeout -k 10 120 python tools/time_ba.py 2>&1 | grep -E "^C4 W 1|^C3" || exit 1
done
