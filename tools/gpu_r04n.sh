#!/bin/bash
# r04: window/BF/BA tests, C1 latencies + trace, io_lat
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/n_tests.log python -u -m pytest tests/test_gpu_window.py tests/test_gpu_bf.py tests/test_gpu_ba.py tests/test_golden.py tests/test_gpu_host_cpp.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/n_c1.log python tools/c1_time.py || exit $?
tools/gpu_step.sh 120 $O/n_iolat.log tools/micro/io_lat || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/n_c1p -o c1 --output-format csv -- python3 $R/tools/c1_time.py > $O/n_c1p.log 2>&1 || exit $?
