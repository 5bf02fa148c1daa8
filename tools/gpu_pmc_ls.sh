#!/bin/bash
# PMC passes over the point-major BA kernels on the 80k-point window (tools/time_ba.py SH80k):
# the available counters, then LDS / VALU / wait counters, one pass each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O/pmc_ls
export TMPDIR=/tmp TIME_BA_ONLY=SH80k
timeout -s KILL 60 rocprofv3 -L > $O/pmc_ls/avail.txt 2>&1
k=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES" \
           "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_BUSY_CYCLES" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmc_ls/p$k -o p$k --output-format csv -- python3 tools/time_ba.py \
    > $O/pmc_ls/p$k.log 2>&1 || echo "pass $k failed rc=$?" >> $O/pmc_ls/fail.txt
done
exit 0
