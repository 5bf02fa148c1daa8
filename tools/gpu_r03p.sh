#!/bin/bash
# r03: Cholesky column-group hand-over: BA parity, then same-box A/B against liblorb_old.so, and the
# per-panel trace (liblorb_trace.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/p_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
for k in 1 2; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/p_time_old_$k.log python tools/time_ba.py || exit $?
  tools/gpu_step.sh 200 $O/p_time_new_$k.log python tools/time_ba.py || exit $?
done
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/p_chol_trace.log python tools/chol_trace.py || exit $?
