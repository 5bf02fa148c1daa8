#!/bin/bash
# r04: back-substitution block trace, then the C4 step A/B (map overlap) + host-phase time + default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/h_trace.log python tools/chol_trace.py || exit $?
tools/gpu_r04e.sh
