#!/bin/bash
# r03: the GPU test files one by one (an ordinary failure does not stop the script; a fault / abort /
# timeout does), smoke, the default bench line, then the round's profiles: kernel stats + FETCH/WRITE
# passes for the C4 chained step and the shared window (tools/pmc_traffic.py), one SQ MFMA pass, and
# the SURVEY 8f row kernels (tools/time_rows.py, incl. the ORB extraction).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
TESTS=${TESTS:-"test_gpu_solver test_gpu_map test_gpu_ba test_gpu_host_cpp"}
fail=0
if [ -n "$CHOL" ]; then  # Cholesky timing and the per-panel trace (tools/build_variant.sh trace -DLORB_CHOL_TRACE)
  tools/gpu_step.sh 200 $O/d_time_ba.log python tools/time_ba.py || exit $?
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/d_chol_trace.log python tools/chol_trace.py || exit $?
fi
for t in $TESTS; do
  tools/gpu_step.sh 300 $O/d_$t.log python -u -m pytest tests/$t.py -m gpu -q --timeout 200 --timeout-method thread
  rc=$?
  [ $rc -gt 1 ] && exit $rc
  [ $rc -ne 0 ] && fail=1
done
tools/gpu_step.sh 120 $O/d_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
rc=$?; [ $rc -gt 1 ] && exit $rc
tools/gpu_step.sh 300 $O/d_bench.log python bench.py
rc=$?; [ $rc -gt 1 ] && exit $rc
[ -n "$NO_PROF" ] && exit $fail
for spec in "c4_chain:c4:--no-c2 --no-dropin --no-shared" "shared_w1:shared:"; do
  key=${spec%%:*}; rest=${spec#*:}; wl=${rest%%:*}; extra=${rest#*:}
  B="$R/bench.py --workload $wl --no-cpu-baseline $extra"
  tools/gpu_step.sh 300 $O/d_prof_${key}_stats.log rocprofv3 --kernel-trace --stats -d $P/$key/stats -o r03_${key} \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
  tools/gpu_step.sh 120 $O/d_prof_${key}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/$key/fetch -o r03_${key}_fetch \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  tools/gpu_step.sh 120 $O/d_prof_${key}_write.log rocprofv3 --pmc WRITE_SIZE -d $P/$key/write -o r03_${key}_write \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  python tools/pmc_traffic.py $P/$key $O/r03_traffic.json --workload $key > $O/d_traffic_$key.log 2>&1 || exit 1
done
tools/gpu_step.sh 120 $O/d_pmc_mfma.log rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_BUSY_CYCLES SQ_WAVES -d $P/mfma -o r03_mfma --output-format csv \
  -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c2 --no-dropin --no-shared || exit $?
tools/gpu_step.sh 300 $O/d_prof_rows.log rocprofv3 --kernel-trace --stats -d $P/rows -o r03_rows --output-format csv \
  -- python3 $R/tools/time_rows.py || exit $?
tools/gpu_step.sh 300 $O/d_rows.log python3 tools/time_rows.py || exit $?
exit $fail
