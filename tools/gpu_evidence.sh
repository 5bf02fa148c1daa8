#!/bin/bash
# A round's GPU evidence, one parameterised runner: tools/gpu_evidence.sh ROUND (e.g. r05).
#   the GPU test files one by one (an ordinary failure does not stop the script; a fault / abort /
#   timeout does), smoke, the default bench line, then the profiles: kernel stats + FETCH / WRITE
#   passes (tools/pmc_traffic.py -> gpurun_out/ROUND_traffic.json) for the C4 chained step, the shared
#   window, C3 and C2, and one SQ MFMA pass.
# Switches: NO_TESTS, NO_BENCH, NO_PROF=1 skip a part; TESTS="test_gpu_x ..." narrows the tests;
# WORKLOADS="c4_chain shared_w1 c3 c2 c4x8" narrows the profiled workloads; TRACE=1 adds the Cholesky trace
# (needs variants/liblorb_trace.so: tools/build_variant.sh trace -DLORB_CHOL_TRACE); C1=1 the C1 trace.
RD=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof_$RD
mkdir -p $O $P
export TMPDIR=/tmp
TESTS=${TESTS:-"test_gpu_solver test_gpu_map test_gpu_ba test_gpu_host_cpp test_gpu_window test_gpu_bf test_gpu_shard test_compute_descriptor test_golden"}
WORKLOADS=${WORKLOADS:-"c4_chain shared_w1 c3 c2 c4x8"}
fail=0
if [ -z "$NO_TESTS" ]; then
  for t in $TESTS; do
    tools/gpu_step.sh 300 $O/${RD}_$t.log python -u -m pytest tests/$t.py -m gpu -q --timeout 200 --timeout-method thread
    rc=$?
    [ $rc -gt 1 ] && exit $rc
    [ $rc -ne 0 ] && fail=1
  done
  tools/gpu_step.sh 120 $O/${RD}_smoke.log python -c "import __graft_entry__ as g; g.smoke()"
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  tools/gpu_step.sh 400 $O/${RD}_bench.log python bench.py
  rc=$?; [ $rc -gt 1 ] && exit $rc
fi
[ -n "$NO_PROF" ] && exit $fail
if [ -n "$TRACE" ]; then
  LORB_LIB_PATH=$R/variants/liblorb_trace.so tools/gpu_step.sh 120 $O/${RD}_chol_trace.log python tools/chol_trace.py || exit $?
fi
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-c4x8"
for key in $WORKLOADS; do
  case $key in
    c4_chain) wl=c4; extra=$NOSUB ;;
    c4x8) wl=c4; extra="$NOSUB --windows 8" ;;
    shared_w1) wl=shared; extra= ;;
    *) wl=$key; extra= ;;
  esac
  B="$R/bench.py --workload $wl --no-cpu-baseline $extra"
  tools/gpu_step.sh 300 $O/${RD}_prof_${key}_stats.log rocprofv3 --kernel-trace --stats -d $P/$key/stats -o ${RD}_${key} \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
  tools/gpu_step.sh 120 $O/${RD}_prof_${key}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/$key/fetch -o ${RD}_${key}_fetch \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  tools/gpu_step.sh 120 $O/${RD}_prof_${key}_write.log rocprofv3 --pmc WRITE_SIZE -d $P/$key/write -o ${RD}_${key}_write \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  python tools/pmc_traffic.py $P/$key $O/${RD}_traffic.json --workload $key > $O/${RD}_traffic_$key.log 2>&1 || exit 1
done
if [ -z "$NO_MFMA" ]; then
  tools/gpu_step.sh 120 $O/${RD}_pmc_mfma.log rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_BUSY_CYCLES SQ_WAVES -d $P/mfma -o ${RD}_mfma --output-format csv \
    -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline $NOSUB || exit $?
fi
if [ -n "$C1" ]; then
  tools/gpu_step.sh 300 $O/${RD}_prof_c1.log rocprofv3 --kernel-trace --memory-copy-trace --stats -d $P/c1 -o ${RD}_c1 \
    --output-format csv -- python3 $R/tools/c1_time.py || exit $?
fi
exit $fail
