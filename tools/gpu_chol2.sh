#!/bin/bash
# Cholesky iteration: BA parity tests, BA timing, per-wave stamps and chain phase cycles
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/q_tests.log python -u -m pytest tests/test_gpu_ba.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/q_time_new.log python tools/time_ba.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_stamps.so tools/gpu_step.sh 120 $O/q_stamps.log python tools/chol_stamps.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_phases.so tools/gpu_step.sh 120 $O/q_phases.log python tools/chol_stamps.py || exit $?
