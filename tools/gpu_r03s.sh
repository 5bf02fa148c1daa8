#!/bin/bash
# r03: ORB extraction evidence on the committed kernels: device time per frame
# (tools/time_orb.py) and the per-kernel split under rocprofv3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O/prof_s
export TMPDIR=/tmp
tools/gpu_step.sh 200 $O/s_orb.log python tools/time_orb.py || exit $?
tools/gpu_step.sh 200 $O/s_orb_prof.log rocprofv3 --kernel-trace --stats -d $O/prof_s/orb -o orb --output-format csv \
  -- python3 $R/tools/time_orb.py --frames 100 || exit $?
