#!/bin/bash
# copy the evidence of tools/gpu_r04_prof.sh (gpurun_out/) into profiles/r04/
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out; P=$O/prof4; D=profiles/r04
mkdir -p $D
grep '^{' $O/p_bench.log | tail -n 1 > $D/bench_default.json
for k in c4_chain shared_w1 c3 c2; do
  cp $P/$k/stats/r04_${k}_kernel_stats.csv $D/${k}_kernel_stats.csv
done
cp $P/c1/r04_c1_kernel_stats.csv $D/c1_kernel_stats.csv
cp $O/r04_traffic.json $D/traffic.json
cp $P/mfma/r04_mfma_counter_collection.csv $D/c4_mfma_pmc.csv
cp $O/p_chol_trace.log $D/chol_trace.log
for f in $O/p_test_*.log $O/p_smoke.log; do echo "== $(basename $f)"; tail -n 3 $f; done > $D/gpu_tests_tail.log
