#!/bin/bash
# r04: chunked Schur -- BA/shard tests, C4 line, shared line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 400 $O/r_tests.log python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_map.py tests/test_gpu_solver.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh 200 $O/r_c4.log python bench.py --no-cpu-baseline --no-c2 --no-dropin --no-shared --no-c3 --no-c1 --steps 200 --warmup 10 || exit $?
tools/gpu_step.sh 300 $O/r_shared.log python bench.py --workload shared --no-cpu-baseline --steps 20 --warmup 3 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r_prof -o sh --output-format csv -- python3 $R/bench.py --workload shared --no-cpu-baseline --steps 5 --warmup 2 > $O/r_prof.log 2>&1 || exit $?
