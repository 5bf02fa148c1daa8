#!/bin/bash
# Same-box A/B of variant libraries (variants/liblorb_<v>.so, tools/build_variant.sh) on the default
# C4 chained step (VARIANTS="a b c", WL="c4 shared c3", ROUNDS=2): ms/step per run into abv_summary.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-c4x8 --no-cpu-baseline"
for r in $(seq ${ROUNDS:-2}); do
  for wl in ${WL:-c4}; do
    for v in $VARIANTS; do
      LORB_LIB_PATH=$R/variants/liblorb_$v.so tools/gpu_step.sh 200 $O/abv_${v}_${wl}_$r.log python bench.py --workload $wl $NOSUB --steps ${STEPS:-30} || exit $?
      python - "$O/abv_${v}_${wl}_$r.log" "$v" "$wl" >> $O/abv_summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print(sys.argv[2], sys.argv[3], "value %.1f ms_per_step %.4f" % (d["value"], d["ms_per_step"]))
PY
    done
  done
done
