#!/bin/bash
# r03: Cholesky pivot on uniform values: BA / map / solver parity, then same-box A/B of the solve
# (tools/time_ba.py) and of the C4 step against liblorb_old.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/g_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
for k in 1 2; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/g_time_old_$k.log python tools/time_ba.py || exit $?
  tools/gpu_step.sh 200 $O/g_time_new_$k.log python tools/time_ba.py || exit $?
done
