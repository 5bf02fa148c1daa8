#!/bin/bash
# r04: Cholesky trace (bottom init preloaded), BA tests, BA timings, C4 line x2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/q_trace.log python tools/chol_trace.py || exit $?
tools/gpu_step.sh 400 $O/q_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_shard.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/q_tba.log python tools/time_ba.py || exit $?
B="python bench.py --no-cpu-baseline --no-c2 --no-dropin --no-shared --no-c3 --no-c1 --steps 200 --warmup 10"
for i in 1 2; do tools/gpu_step.sh 200 $O/q_c4_$i.log $B || exit $?; done
