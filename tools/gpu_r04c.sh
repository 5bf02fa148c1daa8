#!/bin/bash
# r04: chain-delta Cholesky variant (liblorb_cd.so): BA/map/shard/solver parity, trace, timing A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_cd.so tools/gpu_step.sh 400 $O/c_tests_cd.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_tracecd.so tools/gpu_step.sh 120 $O/c_trace_cd.log python tools/chol_trace.py || exit $?
for k in 1 2; do
tools/gpu_step.sh 200 $O/c_tba_def$k.log python tools/time_ba.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_cd.so tools/gpu_step.sh 200 $O/c_tba_cd$k.log python tools/time_ba.py || exit $?
done
