import sys, time, argparse
sys.path.insert(0, '/root/repo' if len(sys.argv) < 2 else sys.argv[1])
import bench
from lorb_slam_amd.runtime import Context
ctx = Context(0)
a = argparse.Namespace(windows=8, steps=20, warmup=3, cpu_budget=1.0)
wl = bench.workload_c4(ctx, a, 0)
maps_step = wl["step"]
for _ in range(3): maps_step()
wl["sync"]()
# time per-map host calls inside step: monkeypatch via closure is hard; time whole steps and per call
import numpy as np
T = []
for _ in range(10):
    t0 = time.perf_counter(); maps_step(); T.append(time.perf_counter() - t0)
wl["sync"]()
print("host time per 8-window step (ms): med %.3f" % (np.median(T) * 1e3), flush=True)
t0 = time.perf_counter()
for _ in range(10): maps_step()
wl["sync"]()
print("wall per step (ms): %.3f" % ((time.perf_counter() - t0) / 10 * 1e3), flush=True)
wl["cleanup"]()
