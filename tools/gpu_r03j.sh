#!/bin/bash
# r03: k_ba_sc (Schur + Cholesky in one launch) parity, then A/B against LORB_NO_SC=1 (separate launches)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/j_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/j_time_sc.log python tools/time_ba.py || exit $?
LORB_NO_SC=1 tools/gpu_step.sh 200 $O/j_time_nosc.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/j_bench_sc.log python bench.py --no-cpu-baseline --no-c2 --no-shared || exit $?
LORB_NO_SC=1 tools/gpu_step.sh 200 $O/j_bench_nosc.log python bench.py --no-cpu-baseline --no-c2 --no-shared || exit $?
tools/gpu_step.sh 200 $O/j_bench_sc2.log python bench.py --no-cpu-baseline --no-c2 --no-shared || exit $?
