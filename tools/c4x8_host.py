"""Diagnostics: the 8-window chained step (bench.py's c4x8 sub-record) timed from the host: host
time per 8-window step and wall time per step.  --torch imports torch and counts devices first (as
bench.py does); --headline runs 30 single-window steps on the same context first."""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--torch", action="store_true")
ap.add_argument("--headline", action="store_true")
ap.add_argument("--close", action="store_true", help="close the headline map before the 8 windows")
ap.add_argument("--twice", action="store_true", help="the 8-window measurement twice (new maps)")
a0 = ap.parse_args()
if a0.torch:
    from lorb_slam_amd.runtime import device_count
    print("devices", device_count(), flush=True)
from lorb_slam_amd.runtime import Context  # noqa: E402
ctx = Context(0)
if a0.headline:
    h = bench.workload_c4(ctx, argparse.Namespace(windows=1, steps=30, warmup=3, cpu_budget=1.0), 0)
    for _ in range(30):
        h["step"]()
    h["sync"]()
    if a0.close:
        h["cleanup"]()
for rep in range(2 if a0.twice else 1):
    a = argparse.Namespace(windows=8, steps=20, warmup=3, cpu_budget=1.0)
    wl = bench.workload_c4(ctx, a, 0)
    for _ in range(3):
        wl["step"]()
    wl["sync"]()
    T = []
    for _ in range(10):
        t0 = time.perf_counter(); wl["step"](); T.append(time.perf_counter() - t0)
    wl["sync"]()
    print("host time per 8-window step (ms): med %.3f" % (np.median(T) * 1e3), flush=True)
    t0 = time.perf_counter()
    for _ in range(10):
        wl["step"]()
    wl["sync"]()
    print("wall per step (ms): %.3f" % ((time.perf_counter() - t0) / 10 * 1e3), flush=True)
    wl["cleanup"]()
