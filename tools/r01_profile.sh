#!/bin/bash
# GPU-box profiling pass for the round: GPU tests, default bench, rocprofv3 --kernel-trace --stats
# of the bench, and two separate PMC passes (FETCH_SIZE / WRITE_SIZE).  Every GPU step has its own
# time limit; the script stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=$R/gpurun_out
P=$O/prof
mkdir -p "$P"
TAG=${1:-r01}
STEPS=${STEPS:-10}
tools/gpu_step.sh 900 $O/tests_gpu.log python -m pytest tests -m gpu -q -x || exit $?
tools/gpu_step.sh 300 $O/bench.log python bench.py || exit $?
tools/gpu_step.sh 300 $O/prof_stats.log rocprofv3 --kernel-trace --stats -d $P/stats -o ${TAG}_c4 \
  --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $O/pmc_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o ${TAG}_c4_fetch \
  --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
tools/gpu_step.sh 300 $O/pmc_write.log rocprofv3 --pmc WRITE_SIZE -d $P/write -o ${TAG}_c4_write \
  --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit $?
python tools/pmc_traffic.py $P $O/${TAG}_traffic.json > $O/traffic.log 2>&1
tools/gpu_step.sh 300 $O/bench_c2.log python bench.py --workload c2 --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh 300 $O/bench_shared.log python bench.py --workload shared --steps 5 --warmup 1 || exit $?
tools/gpu_step.sh 300 $O/prof_shared.log rocprofv3 --kernel-trace --stats -d $P/stats_shared -o ${TAG}_shared \
  --output-format csv -- python3 $R/bench.py --workload shared --steps 5 --warmup 1 --no-cpu-baseline || exit $?
