#!/bin/bash
# r04: C4 Cholesky A/B, default library vs a variant (LORB_LIB_PATH), kernel stats each, twice
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; P=$O/prof_w; mkdir -p $O $P
export TMPDIR=/tmp
V=${V:-nopre}
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1"
for i in 1 2; do
tools/gpu_step.sh 300 $O/w_def$i.log rocprofv3 --kernel-trace --stats -d $P/def$i -o w --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline $NOSUB --steps 10 --warmup 2 || exit $?
LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$V.so tools/gpu_step.sh 300 $O/w_var$i.log rocprofv3 --kernel-trace --stats -d $P/var$i -o w --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline $NOSUB --steps 10 --warmup 2 || exit $?
done
for f in $(find $P -name "*kernel_stats.csv" | sort); do echo "$f $(grep 'k_ba_chol_2s<true>' $f | cut -d, -f4)"; done > $O/w_summary.txt
