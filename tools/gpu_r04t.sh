#!/bin/bash
# r04: back-substitution as w - G y_M (LORB_BSG): BA / solver / shard tests, bench, Cholesky trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 400 $O/t_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $O/t_bench.log python bench.py --no-c1 || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/t_chol_trace.log python tools/chol_trace.py || exit $?
