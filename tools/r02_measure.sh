#!/bin/bash
# Round-2 measurement pass (no profiler): the shared window on RCCL world 1, BA-only solves
# (C3 / C4 / 8 x C4), and the SURVEY §8f rows; each step with its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
tools/gpu_step.sh 300 $O/m_shared.log python bench.py --workload shared --steps 10 --warmup 2 --no-cpu-baseline || exit $?
tools/gpu_step.sh 200 $O/m_time_ba.log python tools/time_ba.py || exit $?
tools/gpu_step.sh 300 $O/m_rows.log python tools/time_rows.py || exit $?
