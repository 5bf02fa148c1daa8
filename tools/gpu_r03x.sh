#!/bin/bash
# r03: k_db_gather column-prefix loop unrolled (liblorb_un.so) vs the default build, same box
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
B="bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared --steps 200 --warmup 10"
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_un.so tools/gpu_step.sh 300 $O/y_tests.log python -u -m pytest tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
for k in 1 2 3; do
  tools/gpu_step.sh 200 $O/y_old_$k.log python $B || exit $?
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_un.so tools/gpu_step.sh 200 $O/y_new_$k.log python $B || exit $?
done
