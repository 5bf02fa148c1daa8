#!/bin/bash
# A/B of the default bench (C4) and the C2 bench: liblorb_old.so vs liblorb.so, then the BF tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/abb_old_c4.log python bench.py --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $O/abb_new_c4.log python bench.py --no-cpu-baseline || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/abb_old_c2.log python bench.py --workload c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $O/abb_new_c2.log python bench.py --workload c2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $O/abb_tests.log python -u -m pytest tests/test_gpu_bf.py tests/test_gpu_window.py tests/test_golden.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
