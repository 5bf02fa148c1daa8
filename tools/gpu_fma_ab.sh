#!/bin/bash
# FP64 contraction A/B under rocprofv3: kernel stats of the C4 chained step, C3
# and the shared window with the shipped library (main) and variants/liblorb_nofma.so
# (tools/build_variant.sh nofma -DLORB_NO_CONTRACT), one box, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out/fma_ab; mkdir -p $O
export TMPDIR=/tmp
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-c4x8 --no-cpu-baseline"
for v in main nofma; do
  lib=$R/lorb_slam_amd/liblorb.so; [ "$v" = nofma ] && lib=$R/variants/liblorb_nofma.so
  for wl in c4 c3 shared; do
    extra=$NOSUB; [ "$wl" = c4 ] || extra="--no-cpu-baseline"
    LORB_LIB_PATH=$lib tools/gpu_step.sh 300 $O/${v}_${wl}.log rocprofv3 --kernel-trace --stats -d $O/$v/$wl -o ${v}_${wl} \
      --output-format csv -- python3 $R/bench.py --workload $wl $extra --steps 20 --warmup 3 || exit $?
  done
done
exit 0
