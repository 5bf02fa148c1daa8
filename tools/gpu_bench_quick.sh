#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/bq_c4.log python bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $O/bq_shared.log python bench.py --workload shared --steps 5 --warmup 1 || exit $?
