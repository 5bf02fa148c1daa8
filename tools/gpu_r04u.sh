#!/bin/bash
# r04: Cholesky trace only (trace variant library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/u_chol_trace.log python tools/chol_trace.py || exit $?
