#!/bin/bash
# r04: bs trace after moving the operator loads; host-phase breakdown; BA tests + timings
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/i_trace.log python tools/chol_trace.py || exit $?
tools/gpu_step.sh 400 $O/i_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LORB_HOST_PHASE=1 tools/gpu_step.sh 200 $O/i_hp.log python bench.py --workload c4 --no-cpu-baseline --no-c2 --no-dropin --no-shared --no-c3 --steps 200 --warmup 10 || exit $?
tools/gpu_step.sh 200 $O/i_tba.log python tools/time_ba.py || exit $?
