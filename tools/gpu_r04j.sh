#!/bin/bash
# r04: full GPU suite (one-wave pose-only, strided candidates); C1 call latencies
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 600 $O/j_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/j_c1.log python tools/c1_time.py --cpu || exit $?
