#!/bin/bash
# r04: MFMA operator build + double-buffered operator prefetch: BA/map/solver/shard parity, trace,
# timing vs the r03 build; host I/O latency; FETCH/WRITE calibration
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
tools/gpu_step.sh 400 $O/f_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_map.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/f_trace.log python tools/chol_trace.py || exit $?
for k in 1 2; do
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_base.so tools/gpu_step.sh 200 $O/f_tba_base$k.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 200 $O/f_tba_new$k.log python tools/time_ba.py || exit $?
done
tools/gpu_step.sh 120 $O/f_iolat.log tools/micro/io_lat || exit $?
tools/gpu_step.sh 120 $O/f_fc_fetch.log timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fc/fetch -o fc --output-format csv -- tools/micro/fetch_cal || exit $?
tools/gpu_step.sh 120 $O/f_fc_write.log timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/fc/write -o fc --output-format csv -- tools/micro/fetch_cal || exit $?
