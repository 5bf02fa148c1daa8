#!/bin/bash
# Generic GPU A/B step: optional tests (TESTS), then tools/time_ba.py on each library given
# (main = lorb_slam_amd/liblorb.so, NAME = variants/liblorb_NAME.so), alternating twice; then the C1
# call latencies (C1=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
rc=0
if [ -n "$TESTS" ]; then
  tools/gpu_step.sh 600 $O/ab_tests.log python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
for k in 1 2; do
  for v in "$@"; do
    lib=$R/variants/liblorb_$v.so; [ "$v" = main ] && lib=$R/lorb_slam_amd/liblorb.so
    LORB_LIB_PATH=$lib tools/gpu_step.sh 200 $O/ab_${v}_$k.log python tools/time_ba.py || exit $?
  done
done
if [ -n "$C1" ]; then
  tools/gpu_step.sh 200 $O/ab_c1.log python tools/c1_time.py || exit $?
fi
exit $rc
