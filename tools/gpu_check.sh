#!/bin/bash
# GPU check of the current tree: full GPU test suite, then the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 600 $O/chk_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $O/chk_bench.log python bench.py || exit $?
