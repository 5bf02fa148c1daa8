#!/bin/bash
# GPU box: BA parity tests, Cholesky phase stamps (stamps build) and BA timings -> gpurun_out/
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ba.py > gpurun_out/ba.log 2>&1 || { tail -20 gpurun_out/ba.log; exit 1; }
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_stamps.so timeout -k 10 120 python tools/chol_stamps.py > gpurun_out/st2.log 2>&1 || { tail gpurun_out/st2.log; exit 1; }
timeout -k 10 120 python tools/time_ba.py > gpurun_out/tba.log 2>&1 || { tail gpurun_out/tba.log; exit 1; }
tail -2 gpurun_out/ba.log; tail -3 gpurun_out/st2.log; tail -5 gpurun_out/tba.log
