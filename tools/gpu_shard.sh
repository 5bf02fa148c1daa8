#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 400 $O/s_tests.log python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_ba.py -m gpu -x -v --timeout 200 --timeout-method thread || exit $?
