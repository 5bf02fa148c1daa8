#!/bin/bash
# r04: full GPU suite, BA timings, default C4 line (no sub-records), fused tail A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 600 $O/o_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/o_tba.log python tools/time_ba.py || exit $?
B="python bench.py --no-cpu-baseline --no-c2 --no-dropin --no-shared --no-c3 --no-c1 --steps 200 --warmup 10"
for i in 1 2; do
  tools/gpu_step.sh 200 $O/o_c4_tail_$i.log $B || exit $?
  LORB_NO_TAIL=1 tools/gpu_step.sh 200 $O/o_c4_notail_$i.log $B || exit $?
done
tools/gpu_step.sh 300 $O/o_shared.log python bench.py --workload shared --no-cpu-baseline --steps 20 --warmup 3 || exit $?
