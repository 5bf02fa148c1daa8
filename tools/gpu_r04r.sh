#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_SCHUR_DEBUG=1 tools/gpu_step.sh 300 $O/s_shared.log python bench.py --workload shared --no-cpu-baseline --steps 5 --warmup 2 || exit $?
