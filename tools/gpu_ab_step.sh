#!/bin/bash
# same-box A/B of the C4 chained step: liblorb_old.so vs liblorb.so, alternating bench runs
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
B="bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared --steps 200 --warmup 10"
for k in 1 2 3; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/ab_old_$k.log python $B || exit $?
  tools/gpu_step.sh 200 $O/ab_new_$k.log python $B || exit $?
done
