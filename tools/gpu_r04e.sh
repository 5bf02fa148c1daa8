#!/bin/bash
# r04: C4 step A/B (map overlap on/off, default vs chain-delta build), host-phase time, then the
# default bench line (all sub-records)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
B="bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared --no-c3 --steps 200 --warmup 10"
LORB_HOST_PHASE=1 tools/gpu_step.sh 200 $O/e_hp.log python $B || exit $?
for k in 1 2; do
tools/gpu_step.sh 200 $O/e_ovl1_$k.log python $B || exit $?
LORB_MAP_OVERLAP=0 tools/gpu_step.sh 200 $O/e_ovl0_$k.log python $B || exit $?
done
tools/gpu_step.sh 400 $O/e_bench.log python bench.py || exit $?
