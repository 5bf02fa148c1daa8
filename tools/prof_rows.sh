#!/bin/bash
# rocprofv3 kernel stats of tools/time_rows.py -> gpurun_out/prow/rows_kernel_stats.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/prow
ROWS_N=${ROWS_N:-50} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prow -o rows --output-format csv \
  -- python3 tools/time_rows.py > gpurun_out/prow.log 2>&1
timeout -k 10 300 python3 tools/time_rows.py > gpurun_out/rows.json 2> gpurun_out/rows.err
