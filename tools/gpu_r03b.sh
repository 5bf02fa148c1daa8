#!/bin/bash
# r03: changed-area GPU tests, the whole -m gpu suite, smoke, default bench line, rocprof kernel stats of the C4 step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 400 $O/b_new.log python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_ba.py tests/test_gpu_bf.py tests/test_gpu_shard.py -m gpu -x -v --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 600 $O/b_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/b_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh 300 $O/b_bench.log python bench.py --no-cpu-baseline || exit $?
rm -rf $O/prof_c4
tools/gpu_step.sh 300 $O/b_prof.log rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python bench.py --steps 10 --warmup 3 --no-c2 --no-dropin --no-shared --no-cpu-baseline || exit $?
