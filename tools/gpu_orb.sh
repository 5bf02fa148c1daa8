#!/bin/bash
# GPU: the ORB extractor tests and the golden ORB fixtures.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/orb_tests.log python -u -m pytest tests/test_gpu_window.py tests/test_golden.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "orb" || exit $?
