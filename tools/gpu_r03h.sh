#!/bin/bash
# r03 (re-entry): every -m gpu test, smoke(), the default bench line, C4 chained-step kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out
P=$O/prof3
mkdir -p $O $P
export TMPDIR=/tmp
tools/gpu_step.sh 600 $O/h_tests.log python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread || exit $?
tools/gpu_step.sh 120 $O/h_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh 300 $O/h_bench.log python bench.py || exit $?
rm -rf $P/c4h
tools/gpu_step.sh 300 $O/h_prof.log rocprofv3 --kernel-trace --stats -d $P/c4h -o c4h --output-format csv \
  -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c2 --no-dropin --no-shared || exit $?
