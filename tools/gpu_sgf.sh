#!/bin/bash
# GPU: the shared window with partial runs of F groups (LORB_SG_F, FS="1 3 5 8"): bench line + kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for f in ${FS:-1 3 5 8}; do
  LORB_SG_F=$f tools/gpu_step.sh 200 $O/sgf_$f.log python bench.py --workload shared --no-cpu-baseline --steps 30 || exit $?
  LORB_SG_F=$f tools/gpu_step.sh 200 $O/sgf_prof_$f.log rocprofv3 --kernel-trace --stats -d $O/sgf_prof/f$f -o sgf$f \
    --output-format csv -- python3 $R/bench.py --workload shared --no-cpu-baseline --steps 10 --warmup 2 || exit $?
done
