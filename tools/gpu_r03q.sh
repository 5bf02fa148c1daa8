#!/bin/bash
# r03 step-structure pass: map / solver / BA GPU tests, the C4 chained-step kernel stats, the
# crossCheck scan's chunk-count sweep (LORB_BF_NC, diagnostics knob), and the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof_q
mkdir -p $O $P
export TMPDIR=/tmp
for t in ${TESTS:-test_gpu_map test_gpu_solver test_gpu_ba test_gpu_bf}; do
  tools/gpu_step.sh 300 $O/q_$t.log python -u -m pytest tests/$t.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
done
B="$R/bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared"
for nc in ${NCS:-0 32 64}; do
  LORB_BF_NC=$nc tools/gpu_step.sh 300 $O/q_stats_nc$nc.log rocprofv3 --kernel-trace --stats -d $P/nc$nc -o q_nc$nc \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
done
tools/gpu_step.sh 300 $O/q_bench.log python bench.py --no-cpu-baseline || exit $?
