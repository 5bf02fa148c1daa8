"""C1 per-frame call latencies (a2 / a4 / a12) on the GPU through the C-ABI, as bench.py's C1
sub-record measures them; optional oracle leg (--cpu).  Diagnostic."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from lorb_slam_amd.runtime import Context  # noqa: E402

ctx = Context(0)
r = bench.sub_c1(ctx, bench.Dist(), None)
print(json.dumps(r["stage_ms_median"] if "stage_ms_median" in r else r))
if "--cpu" in sys.argv:
    print(json.dumps(bench.cpu_baseline_c1(4.0)["stage_ms_median"]))
