#!/bin/bash
# r03: the new / changed GPU tests first, then the whole -m gpu suite, smoke and the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
tools/gpu_step.sh 400 $O/a_new.log python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_shard.py tests/test_gpu_host_cpp.py -m gpu -x -v --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 600 $O/a_tests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/a_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh 300 $O/a_bench.log python bench.py --no-cpu-baseline || exit $?
