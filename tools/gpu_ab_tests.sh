#!/bin/bash
# A/B timing of several builds (tools/gpu_abn.sh NAME...), then the BA / shard / map GPU tests on
# the in-tree liblorb.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_abn.sh "$@" || exit $?
tools/gpu_step.sh 400 $O/ab_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_shard.py tests/test_gpu_map.py tests/test_gpu_host_cpp.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
