#!/bin/bash
# GPU box: one SQ PMC pass over the chained C4 bench: wave cycles split into issuing / parked on
# s_waitcnt or a barrier / issue-stalled, per kernel (tools/pmc_sq.py summarises)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/pmcsq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
  -d gpurun_out/pmcsq -o sq --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c2 > gpurun_out/pmcsq.log 2>&1
