#!/bin/bash
# r04: kernel + copy trace of the C1 calls
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/k_c1 -o c1 --output-format csv -- python3 $R/tools/c1_time.py > $O/k_c1.log 2>&1 || exit $?
