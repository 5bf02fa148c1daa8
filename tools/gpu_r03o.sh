#!/bin/bash
# r03: LM iteration tails inside the next k_ba_lin (one launch fewer per iteration): BA / map / solver
# parity, then same-box A/B against LORB_NO_DEC=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/o_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_host_cpp.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/o_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for k in 1 2; do
  LORB_NO_DEC=1 tools/gpu_step.sh 200 $O/o_time_nd_$k.log python tools/time_ba.py || exit $?
  tools/gpu_step.sh 200 $O/o_time_d_$k.log python tools/time_ba.py || exit $?
done
LORB_NO_DEC=1 tools/gpu_step.sh 200 $O/o_bench_nd.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
tools/gpu_step.sh 200 $O/o_bench_d.log python bench.py --no-cpu-baseline --no-c2 --no-shared --no-dropin --steps 50 || exit $?
