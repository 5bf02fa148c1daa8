#!/bin/bash
# copy the evidence of tools/gpu_r03d.sh (gpurun_out/) into profiles/r03/
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; P=$O/prof3; D=profiles/r03
grep '^{' $O/d_bench.log | tail -n 1 > $D/bench_default.json
cp $P/c4_chain/stats/r03_c4_chain_kernel_stats.csv $D/c4_chain_kernel_stats.csv
cp $P/shared_w1/stats/r03_shared_w1_kernel_stats.csv $D/shared_w1_kernel_stats.csv
cp $O/r03_traffic.json $D/traffic.json
cp $P/mfma/r03_mfma_counter_collection.csv $D/c4_mfma_pmc.csv
cp $P/rows/r03_rows_kernel_stats.csv $D/rows_kernel_stats.csv
grep '^{' $O/d_rows.log | tail -n 1 > $D/rows.json
for f in $O/d_test_gpu_*.log $O/d_smoke.log; do echo "== $(basename $f)"; tail -n 3 $f; done > $D/gpu_tests_tail.log
