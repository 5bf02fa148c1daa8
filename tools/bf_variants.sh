#!/bin/bash
# GPU box: BF parity tests, then the C2 bench under LORB_BF_QPL = 1, 2, 4
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bf.py tests/test_gpu_shard.py > gpurun_out/bfv.log 2>&1 || { tail -20 gpurun_out/bfv.log; exit 1; }
tail -1 gpurun_out/bfv.log
for q in 2 4 1; do
  LORB_BF_QPL=$q timeout -k 10 200 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bfv_$q.log 2>&1 || { tail gpurun_out/bfv_$q.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bfv_$q.log').read().strip().splitlines()[-1]); print('QPL=$q', round(d['value']/1e6,1), 'M/s frac', round(d['roofline']['frac'],3), 'us', round(d['roofline']['avg_kernel_us'],1))"
done
