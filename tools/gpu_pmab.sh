#!/bin/bash
# C4 chained-step A/B of the Schur path: bench.py's default workload (no sub-records) with the
# point-major path (LORB_PM=1) and the pair-major one (LORB_PM=0), alternating twice; with
# KT=1 a third pass per path with per-kernel timing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
B="python bench.py --no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-c4x8 --no-cpu-baseline --steps ${STEPS:-100} --warmup 5"
for k in 1 2; do
  for pm in 1 0; do
    LORB_PM=$pm tools/gpu_step.sh 200 $O/pmab_${pm}_$k.log $B || exit $?
  done
done
exit 0
