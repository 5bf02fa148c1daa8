#!/bin/bash
# Point-major BA path check: the BA / map / solver / shard GPU tests, then tools/time_ba.py with the
# point-major path and with the pair-major one (LORB_PM=0), alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
T=${TESTS:-"tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_shard.py tests/test_golden.py"}
tools/gpu_step.sh 600 $O/pm_tests.log python -u -m pytest $T -m gpu -x -v --timeout 200 --timeout-method thread
rc=$?; [ $rc -gt 1 ] && exit $rc
for k in 1 2; do
  tools/gpu_step.sh 200 $O/pm_time_new_$k.log python tools/time_ba.py || exit $?
  LORB_PM=0 tools/gpu_step.sh 200 $O/pm_time_old_$k.log python tools/time_ba.py || exit $?
done
exit $rc
