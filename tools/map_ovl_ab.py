"""Diagnostics: the C4 chained step with the map's overlap on and off, alternating, same process:
wall ms per step over 30 steps (bench.py's workload_c4 maps and keyframe stream)."""
import argparse
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
from lorb_slam_amd.runtime import Context  # noqa: E402

ctx = Context(0)
for rep in range(2):
    for ovl in (True, False):
        a = argparse.Namespace(windows=1, steps=30, warmup=3, cpu_budget=1.0)
        wl = bench.workload_c4(ctx, a, 0)
        for m in wl.get("maps", []):
            m.set_overlap(ovl)
        if "set_overlap" in wl:
            wl["set_overlap"](ovl)
        for _ in range(3):
            wl["step"]()
        wl["sync"]()
        t0 = time.perf_counter()
        for _ in range(30):
            wl["step"]()
        wl["sync"]()
        print("overlap", ovl, "ms/step %.4f" % ((time.perf_counter() - t0) / 30 * 1e3), flush=True)
        wl["cleanup"]()
