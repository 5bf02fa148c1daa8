#!/bin/bash
# r04 final check: every GPU test file in one process, then smoke
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 600 $O/y_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/y_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
