#!/bin/bash
# A/B timing (tools/gpu_abn.sh NAME...) + the whole -m gpu suite on the in-tree liblorb.so + the bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_abn.sh "$@" || exit $?
tools/gpu_step.sh 600 $O/r_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $O/r_bench.log python bench.py --no-cpu-baseline || exit $?
