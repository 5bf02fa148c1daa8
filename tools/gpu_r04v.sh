#!/bin/bash
# r04: C4 chained-step kernel stats only
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; P=$O/prof_v; mkdir -p $O $P
export TMPDIR=/tmp
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1"
tools/gpu_step.sh 300 $O/v_stats.log rocprofv3 --kernel-trace --stats -d $P -o v_c4 --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline $NOSUB --steps 10 --warmup 2 || exit $?
