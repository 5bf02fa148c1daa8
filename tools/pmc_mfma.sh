#!/bin/bash
# GPU box: one SQ PMC pass over the C4 bench (MFMA utilisation of the BA kernels)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/pmcmf
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
  -d gpurun_out/pmcmf -o mf --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcmf.log 2>&1
