#!/bin/bash
# r04 evidence: the GPU test files one by one (an ordinary failure does not stop the script; a fault /
# abort / timeout does), smoke, the default bench line, then the round's profiles: kernel stats +
# FETCH/WRITE passes (tools/pmc_traffic.py -> gpurun_out/r04_traffic.json) for the C4 chained step, the
# shared window, C3 and C2, one SQ MFMA pass, the Cholesky trace and the C1 call trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof4
mkdir -p $O $P
export TMPDIR=/tmp
TESTS=${TESTS:-"test_gpu_solver test_gpu_map test_gpu_ba test_gpu_host_cpp test_gpu_window test_gpu_bf test_gpu_shard test_compute_descriptor test_golden"}
fail=0
if [ -z "$NO_TESTS" ]; then
  for t in $TESTS; do
    tools/gpu_step.sh 300 $O/p_$t.log python -u -m pytest tests/$t.py -m gpu -q --timeout 200 --timeout-method thread
    rc=$?
    [ $rc -gt 1 ] && exit $rc
    [ $rc -ne 0 ] && fail=1
  done
  tools/gpu_step.sh 120 $O/p_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  tools/gpu_step.sh 400 $O/p_bench.log python bench.py
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
[ -n "$NO_PROF" ] && exit $fail
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_trace.so tools/gpu_step.sh 120 $O/p_chol_trace.log python tools/chol_trace.py || exit $?
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1"
for spec in "c4_chain:c4:$NOSUB" "shared_w1:shared:" "c3:c3:" "c2:c2:"; do
  key=${spec%%:*}; rest=${spec#*:}; wl=${rest%%:*}; extra=${rest#*:}
  B="$R/bench.py --workload $wl --no-cpu-baseline $extra"
  tools/gpu_step.sh 300 $O/p_prof_${key}_stats.log rocprofv3 --kernel-trace --stats -d $P/$key/stats -o r04_${key} \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
  tools/gpu_step.sh 120 $O/p_prof_${key}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/$key/fetch -o r04_${key}_fetch \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  tools/gpu_step.sh 120 $O/p_prof_${key}_write.log rocprofv3 --pmc WRITE_SIZE -d $P/$key/write -o r04_${key}_write \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  python tools/pmc_traffic.py $P/$key $O/r04_traffic.json --workload $key > $O/p_traffic_$key.log 2>&1 || exit 1
done
tools/gpu_step.sh 120 $O/p_pmc_mfma.log rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
  SQ_BUSY_CYCLES SQ_WAVES -d $P/mfma -o r04_mfma --output-format csv \
  -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline $NOSUB || exit $?
tools/gpu_step.sh 300 $O/p_prof_c1.log rocprofv3 --kernel-trace --memory-copy-trace --stats -d $P/c1 -o r04_c1 \
  --output-format csv -- python3 $R/tools/c1_time.py || exit $?
exit $fail
