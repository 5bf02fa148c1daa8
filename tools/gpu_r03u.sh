#!/bin/bash
# r03: crossCheck scan lanes per thread (LORB_BF_QPL) on the C4 chained step, kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O/prof_u
export TMPDIR=/tmp
B="$R/bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared"
for q in 1 2 4; do
  LORB_BF_QPL=$q tools/gpu_step.sh 300 $O/u_q$q.log rocprofv3 --kernel-trace --stats -d $O/prof_u/q$q -o u_q$q \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
done
