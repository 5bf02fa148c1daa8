R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_old.so tools/gpu_step.sh 200 $O/ab_old.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/ab_new.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 300 $O/ab_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
