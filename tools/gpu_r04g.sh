#!/bin/bash
# r04: unrolled operator back-substitution: BA parity, trace, timing vs the r03 build
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 400 $O/g_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/g_trace.log python tools/chol_trace.py || exit $?
for k in 1 2; do
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_base.so tools/gpu_step.sh 200 $O/g_tba_base$k.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/g_tba_new$k.log python tools/time_ba.py || exit $?
done
