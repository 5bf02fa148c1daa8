#!/bin/bash
# Cholesky trace + timing A/B + BA parity tests of variant builds: tools/gpu_trace_ab.sh V1 V2 ...
# (liblorb_V.so timed against liblorb_base.so; liblorb_traceV.so traced)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
for v in "$@"; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace$v.so tools/gpu_step.sh 120 $O/tr_trace$v.log python tools/chol_trace.py || exit $?
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so tools/gpu_step.sh 300 $O/ab_tests_$v.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_shard.py tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
done
tools/gpu_abn.sh base "$@" || exit $?
