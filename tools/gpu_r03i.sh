#!/bin/bash
# r03: k_db_sorted (LDS bits, run-local duplicate check) parity + timing; ORB extraction device time
# (rocprof incl. k_orb_octree); map step phase split.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 400 $O/i_tests.log python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_ba.py -m gpu -x -v --timeout 200 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/i_bench.log python bench.py --no-cpu-baseline --no-c2 --no-shared || exit $?
rm -rf $P/c4i
tools/gpu_step.sh 300 $O/i_prof.log rocprofv3 --kernel-trace --stats -d $P/c4i -o c4i --output-format csv \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c2 --no-dropin --no-shared || exit $?
tools/gpu_step.sh 200 $O/i_orb.log python tools/time_orb.py || exit $?
rm -rf $P/orb
tools/gpu_step.sh 200 $O/i_orb_prof.log rocprofv3 --kernel-trace --stats -d $P/orb -o orb --output-format csv \
  -- python3 $R/tools/time_orb.py --frames 50 || exit $?
LORB_MAP_PROFILE=1 tools/gpu_step.sh 200 $O/i_mapprof.log python tools/map_profile.py --steps 20 || exit $?
tools/gpu_step.sh 200 $O/i_map.log python tools/map_profile.py --steps 20 || exit $?
