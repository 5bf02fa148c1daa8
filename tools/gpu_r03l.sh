#!/bin/bash
# r03: k_orb_octree LDS path: ORB parity (bit-exact vs the oracle, golden), then device time per frame
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/l_orb_tests.log python -u -m pytest tests/test_gpu_window.py tests/test_golden.py -m gpu -x -v --timeout 120 --timeout-method thread -k "orb" || exit $?
tools/gpu_step.sh 200 $O/l_orb.log python tools/time_orb.py || exit $?
rm -rf $P/orbl
tools/gpu_step.sh 200 $O/l_orb_prof.log rocprofv3 --kernel-trace --stats -d $P/orbl -o orb --output-format csv \
  -- python3 $R/tools/time_orb.py --frames 50 || exit $?
tools/gpu_step.sh 120 $O/l_oct_stamps.log python tools/oct_stamps.py || exit $?
