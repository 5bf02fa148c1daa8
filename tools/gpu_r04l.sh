#!/bin/bash
# r04: pull-kernel inputs + mapped direct outputs: full GPU suite, C1 latencies, C1 trace
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 600 $O/l_tests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/l_c1.log python tools/c1_time.py || exit $?
tools/gpu_step.sh 120 $O/l_iolat.log tools/micro/io_lat || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/l_c1p -o c1 --output-format csv -- python3 $R/tools/c1_time.py > $O/l_c1p.log 2>&1 || exit $?
