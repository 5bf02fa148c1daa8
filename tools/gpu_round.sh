#!/bin/bash
# Round check: every -m gpu test, smoke(), then the default bench line (what the driver runs).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
tools/gpu_step.sh 600 $O/r_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/r_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh 300 $O/r_bench.log python bench.py || exit $?
