#!/bin/bash
# r04: resolver round counts on the C1 inputs (debug variant library)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_rdbg.so tools/gpu_step.sh 200 $O/t_rdbg.log python -c "
import sys; sys.path.insert(0, '.')
import bench
from lorb_slam_amd.runtime import Context, lib
ctx = Context(0)
xs = bench.c1_inputs()[:4]
for x in xs:
    calls, keep = bench.c1_calls(x, lib(), ctx.handle)
    calls['a4_search_by_projection_th15']()
" || exit $?
