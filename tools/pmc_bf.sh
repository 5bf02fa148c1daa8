#!/bin/bash
# GPU box: one SQ PMC pass over the C2 brute-force workload (k_bf_scan<top2>)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/pmcbf
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  -d gpurun_out/pmcbf -o bf --output-format csv -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcbf.log 2>&1
