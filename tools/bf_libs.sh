#!/bin/bash
# GPU box: BF parity tests + C2 bench for each lorb_slam_amd/liblorb_<v>.so argument
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  export LORB_LIB_PATH=$R/lorb_slam_amd/liblorb_$v.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf.py > gpurun_out/bfl_$v.log 2>&1 || { tail -20 gpurun_out/bfl_$v.log; exit 1; }
  for q in 2 4; do
    LORB_BF_QPL=$q timeout -k 10 200 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bfl_${v}_$q.log 2>&1 || { tail gpurun_out/bfl_${v}_$q.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/bfl_${v}_$q.log').read().strip().splitlines()[-1]); print('$v QPL=$q', round(d['value']/1e6,1), 'M/s frac', round(d['roofline']['frac'],3), 'us', round(d['roofline']['avg_kernel_us'],1))"
  done
done
