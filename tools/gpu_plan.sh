#!/bin/bash
# BA/map GPU parity tests, then the chained-step timing (plain and per-phase) and the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 400 $O/plan_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/plan_prof.log python tools/map_profile.py --steps 20 || exit $?
LORB_MAP_PROFILE=1 tools/gpu_step.sh 120 $O/plan_prof_phases.log python tools/map_profile.py --steps 20 || exit $?
tools/gpu_step.sh 300 $O/plan_bench.log python bench.py --no-cpu-baseline --no-c2 || exit $?
