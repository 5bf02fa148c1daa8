#!/bin/bash
# GPU check of the current tree, BA-first: the BA / solver / map tests, then the rest of the GPU
# suite, then the default bench line (tools/gpu_step.sh stops the script on a fault / timeout).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/g1_ba.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_map.py -m gpu -v --timeout 200 --timeout-method thread
rc=$?; [ $rc -gt 1 ] && exit $rc
tools/gpu_step.sh 400 $O/g1_rest.log python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_ba.py --deselect tests/test_gpu_solver.py --deselect tests/test_gpu_map.py
rc2=$?; [ $rc2 -gt 1 ] && exit $rc2
tools/gpu_step.sh 300 $O/g1_bench.log python bench.py || exit $?
exit $(( rc | rc2 ))
