#!/bin/bash
# Same-box A/B of variant libraries (variants/liblorb_<v>.so) on the C4 headline AND the 8-window
# sub-record (map groups, one plan of 8, four plans of 2): VARIANTS="a b", ROUNDS=2 -> abx8_summary.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=$R/gpurun_out; mkdir -p $O
NOSUB="--no-c2 --no-dropin --no-shared --no-c3 --no-c1 --no-cpu-baseline"
for r in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    LORB_LIB_PATH=$R/variants/liblorb_$v.so tools/gpu_step.sh 300 $O/abx8_${v}_$r.log python bench.py $NOSUB --steps ${STEPS:-100} || exit $?
    python - "$O/abx8_${v}_$r.log" "$v" >> $O/abx8_summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); x = d.get("c4x8") or {}; op = x.get("one_plan") or {}
        print(sys.argv[2], "c4 %.1f (%.4f ms)  c4x8 %.0f  one_plan %.0f  four_plans_x2 %.0f" % (
            d["value"], d["ms_per_step"], x.get("value", 0), op.get("value", 0), (op.get("four_plans_x2") or {}).get("value", 0)))
PY
  done
done
