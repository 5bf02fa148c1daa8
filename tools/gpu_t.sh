#!/bin/bash
# GPU: the named test files only (TESTS="tests/a.py tests/b.py"), verbose, under the step limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh ${SECS:-300} $O/t_${TAG:-run}.log python -u -m pytest $TESTS -m gpu -v --timeout 200 --timeout-method thread
