#!/bin/bash
# r04 baseline on this round's box: Cholesky trace (trace build), BA timings, GPU suite
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/a_trace.log python tools/chol_trace.py || exit $?
tools/gpu_step.sh 200 $O/a_tba.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 600 $O/a_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
