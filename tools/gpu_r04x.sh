#!/bin/bash
# r04: C4 Cholesky A/B over variant libraries (default, then each of $VS), kernel stats, twice;
# the BA / solver / map GPU tests on the last variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; P=$O/prof_x; mkdir -p $O $P
export TMPDIR=/tmp
VS=${VS:-"spin ffix"}
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1"
for v in $VS; do
  LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so tools/gpu_step.sh 300 $O/x_t_$v.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_solver.py tests/test_gpu_map.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
done
for i in 1 2; do
  for v in def $VS; do
    L=""; [ $v != def ] && L=$R/lorb_slam_amd/liblorb_$v.so
    LORB_LIB_PATH=$L tools/gpu_step.sh 300 $O/x_$v$i.log rocprofv3 --kernel-trace --stats -d $P/$v$i -o x --output-format csv -- python3 $R/bench.py --workload c4 --no-cpu-baseline $NOSUB --steps 10 --warmup 2 || exit $?
  done
done
for f in $(find $P -name "*kernel_stats.csv" | sort); do echo "$f $(grep 'k_ba_chol_2s<true>' $f | cut -d, -f4) $(grep 'k_ba_lin(' $f | cut -d, -f4)"; done > $O/x_summary.txt
