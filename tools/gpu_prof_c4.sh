#!/bin/bash
# rocprofv3 kernel stats of the chained C4 step (bench c4 workload), into gpurun_out/prof_c4/
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=$R/gpurun_out; mkdir -p $O/prof_c4
tools/gpu_step.sh 300 $O/prof_c4.log rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 --output-format csv -- \
  python3 $R/bench.py --workload c4 --no-cpu-baseline --no-c2 --steps 10 --warmup 2 || exit $?
