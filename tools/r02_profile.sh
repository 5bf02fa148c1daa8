#!/bin/bash
# Round-2 profiling pass: per workload (c4 chained step, c2, shared window on RCCL world 1) one
# rocprofv3 --kernel-trace --stats run and two separate PMC runs (FETCH_SIZE, WRITE_SIZE), then
# tools/pmc_traffic.py merges each into one traffic.json keyed by workload.  Every GPU step has its
# own time limit; the script stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=$R/gpurun_out
P=$O/prof
mkdir -p "$P"
TAG=${1:-r02}
for spec in "c4_chain:c4:--no-c2" "c2:c2:" "shared_w1:shared:"; do
  key=${spec%%:*}; rest=${spec#*:}; wl=${rest%%:*}; extra=${rest#*:}
  B="$R/bench.py --workload $wl --no-cpu-baseline $extra"
  tools/gpu_step.sh 300 $O/prof_${key}_stats.log rocprofv3 --kernel-trace --stats -d $P/$key/stats -o ${TAG}_${key} \
    --output-format csv -- python3 $B --steps 10 --warmup 2 || exit $?
  tools/gpu_step.sh 120 $O/prof_${key}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $P/$key/fetch -o ${TAG}_${key}_fetch \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  tools/gpu_step.sh 120 $O/prof_${key}_write.log rocprofv3 --pmc WRITE_SIZE -d $P/$key/write -o ${TAG}_${key}_write \
    --output-format csv -- python3 $B --steps 3 --warmup 1 || exit $?
  python tools/pmc_traffic.py $P/$key $O/${TAG}_traffic.json --workload $key > $O/traffic_$key.log 2>&1 || exit 1
done
