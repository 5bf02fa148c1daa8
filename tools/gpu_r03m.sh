#!/bin/bash
# r03: fused LM iteration 0 (BA/map/solver parity, BA timing, bench) and the ORB octree LDS path
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/m_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_host_cpp.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 300 $O/m_orb_tests.log python -u -m pytest tests/test_gpu_window.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -k orb || exit $?
tools/gpu_step.sh 200 $O/m_time_ba.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/m_bench.log python bench.py --no-cpu-baseline --no-c2 --no-shared || exit $?
tools/gpu_step.sh 200 $O/m_orb.log python tools/time_orb.py || exit $?
tools/gpu_step.sh 120 $O/m_oct_stamps.log python tools/oct_stamps.py || exit $?
