#!/bin/bash
# r03: Cholesky A/B (tools/build_variant.sh: linv = -DLORB_LINV67, bsrl = -DLORB_BS_RL, linvrl = both)
# with per-panel traces, then the profile passes gpu_r03d.sh did not reach.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 300 $O/f_test_ba.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py -m gpu -q --timeout 200 --timeout-method thread || exit $?
for v in base linv bsrl linvrl; do
  L=$R/lorb_slam_amd/liblorb_$v.so; [ $v = base ] && L=$R/lorb_slam_amd/liblorb.so
  LORB_LIB_PATH=$L tools/gpu_step.sh 200 $O/f_time_$v.log python tools/time_ba.py || exit $?
done
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_linvrl_trace.so tools/gpu_step.sh 120 $O/f_trace_linvrl.log python tools/chol_trace.py || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_linvrl.so tools/gpu_step.sh 300 $O/f_test_ba_linvrl.log python -u -m pytest tests/test_gpu_ba.py -m gpu -q --timeout 200 --timeout-method thread || exit $?
[ -n "$NO_PROF" ] && exit 0
key=shared_w1; B="$R/bench.py --workload shared --no-cpu-baseline"
tools/gpu_step.sh 120 $O/f_prof_${key}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/$key/fetch -o r03_${key}_fetch \
  --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
tools/gpu_step.sh 120 $O/f_prof_${key}_write.log rocprofv3 --pmc WRITE_SIZE -d $P/$key/write -o r03_${key}_write \
  --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
python tools/pmc_traffic.py $P/$key $O/r03_traffic.json --workload $key > $O/f_traffic_$key.log 2>&1 || exit 1
tools/gpu_step.sh 120 $O/f_pmc_mfma.log rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_BUSY_CYCLES SQ_WAVES -d $P/mfma -o r03_mfma --output-format csv \
  -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c2 --no-dropin --no-shared || exit $?
tools/gpu_step.sh 300 $O/f_prof_rows.log rocprofv3 --kernel-trace --stats -d $P/rows -o r03_rows --output-format csv \
  -- python3 $R/tools/time_rows.py || exit $?
tools/gpu_step.sh 300 $O/f_rows.log python3 tools/time_rows.py || exit $?
