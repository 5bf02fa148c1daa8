#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
export TMPDIR=/tmp
O=$R/gpurun_out/pmc; mkdir -p $O
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "k_ba_(chol|schur)" -d $O/p$i -o pmc$i --output-format csv -- python3 $R/tools/prof_ba.py > $O/p$i.log 2>&1 || exit 1
done
