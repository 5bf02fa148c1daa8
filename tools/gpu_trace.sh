#!/bin/bash
# Kernel timeline of the C4 chained step (rocprofv3 --kernel-trace, csv) and its gap analysis
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-c4x8 --no-cpu-baseline"
tools/gpu_step.sh 200 $O/trace_run.log rocprofv3 --kernel-trace -d $O/trace -o c4 --output-format csv \
  -- python3 $R/bench.py --steps 20 --warmup 3 $NOSUB || exit $?
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $f > $O/trace_gaps.txt 2>&1
