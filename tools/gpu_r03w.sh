#!/bin/bash
# r03: crossCheck merge at the head of the append: map / bf / solver parity, kernel stats, and the
# same-box A/B of the C4 step against liblorb_old.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O/prof_x
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/x_tests.log python -u -m pytest tests/test_gpu_map.py tests/test_gpu_bf.py tests/test_gpu_solver.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
B="bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared"
tools/gpu_step.sh 300 $O/x_stats.log rocprofv3 --kernel-trace --stats -d $O/prof_x/s -o x --output-format csv \
  -- python3 $R/$B --steps 10 --warmup 2 || exit $?
for k in 1 2 3; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/x_old_$k.log python $B --steps 200 --warmup 10 || exit $?
  tools/gpu_step.sh 200 $O/x_new_$k.log python $B --steps 200 --warmup 10 || exit $?
done
