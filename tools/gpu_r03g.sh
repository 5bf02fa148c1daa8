#!/bin/bash
# r03: BA/map/solver/shard parity, BA timing + Cholesky trace, the default bench line, C4 kernel stats
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/g_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_shard.py -m gpu -q --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/g_time_ba.log python tools/time_ba.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/g_chol_trace.log python tools/chol_trace.py || exit $?
tools/gpu_step.sh 300 $O/g_bench.log python bench.py --no-cpu-baseline || exit $?
rm -rf $P/c4g
tools/gpu_step.sh 300 $O/g_prof.log rocprofv3 --kernel-trace --stats -d $P/c4g -o c4g --output-format csv \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c2 --no-dropin --no-shared || exit $?
