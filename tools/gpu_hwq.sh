#!/bin/bash
# c4x8 (8 chained C4 windows, one stream each) against the HIP hardware-queue count per process
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
for q in 4 8 16 4 8 16; do
  GPU_MAX_HW_QUEUES=$q tools/gpu_step.sh 120 $O/hwq_$q.log python tools/c4x8_host.py || exit $?
  echo "q=$q $(grep wall $O/hwq_$q.log)" >> $O/hwq_summary.txt
done
