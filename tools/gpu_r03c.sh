#!/bin/bash
# r03: GPU test files one by one (an ordinary failure does not stop the script; a fault / abort /
# timeout does), then smoke, the default bench line and the rocprof kernel stats of the C4 step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
fail=0
for t in test_gpu_solver test_gpu_map test_gpu_ba test_gpu_shard test_gpu_bf test_gpu_window test_gpu_host_cpp; do
  tools/gpu_step.sh 300 $O/c_$t.log python -u -m pytest tests/$t.py -m gpu -q --timeout 200 --timeout-method thread
  rc=$?
  [ $rc -gt 1 ] && exit $rc
  [ $rc -ne 0 ] && fail=1
done
tools/gpu_step.sh 600 $O/c_rest.log python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_solver.py --deselect tests/test_gpu_map.py --deselect tests/test_gpu_ba.py --deselect tests/test_gpu_shard.py --deselect tests/test_gpu_bf.py --deselect tests/test_gpu_window.py --deselect tests/test_gpu_host_cpp.py
rc=$?; [ $rc -gt 1 ] && exit $rc
tools/gpu_step.sh 120 $O/c_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
rc=$?; [ $rc -gt 1 ] && exit $rc
tools/gpu_step.sh 300 $O/c_bench.log python bench.py --no-cpu-baseline
rc=$?; [ $rc -gt 1 ] && exit $rc
rm -rf $O/prof_c4
tools/gpu_step.sh 300 $O/c_prof.log rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python bench.py --steps 10 --warmup 3 --no-c2 --no-dropin --no-shared --no-cpu-baseline
exit $fail
