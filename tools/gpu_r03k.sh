#!/bin/bash
# r03: k_ba_sc variants: coherent loads (default) vs acquire-fence + plain loads (liblorb_scinv.so) vs
# separate launches (LORB_NO_SC=1); parity of the scinv variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_scinv.so tools/gpu_step.sh 300 $O/k_tests_inv.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LORB_NO_SC=1 tools/gpu_step.sh 200 $O/k_time_nosc.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/k_time_sc.log python tools/time_ba.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_scinv.so tools/gpu_step.sh 200 $O/k_time_inv.log python tools/time_ba.py || exit $?
