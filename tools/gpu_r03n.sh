#!/bin/bash
# r03: same-box A/B of the fused LM iteration 0 (LORB_NO_FUSE0=1: iteration 0 unfused), BA timing + bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  LORB_NO_FUSE0=1 tools/gpu_step.sh 200 $O/n_time_nf0_$k.log python tools/time_ba.py || exit $?
  tools/gpu_step.sh 200 $O/n_time_f0_$k.log python tools/time_ba.py || exit $?
done
LORB_NO_FUSE0=1 tools/gpu_step.sh 200 $O/n_bench_nf0.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
tools/gpu_step.sh 200 $O/n_bench_f0.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
LORB_NO_FUSE0=1 tools/gpu_step.sh 200 $O/n_bench_nf0b.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
tools/gpu_step.sh 200 $O/n_bench_f0b.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
