"""Quick GPU timing of the local-BA plan (C3 / C4 / 8 x C4 / the 80k-point shared window), 10 LM
iterations, tolerances 0; per-kernel ms of the linearisation (k_ba_ls), the partial reduction
(k_ba_red) and the Cholesky."""
import sys, os, time, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from lorb_slam_amd import synth, _abi as A
from lorb_slam_amd.runtime import Context, BAPlan, lib
ctx = Context(0)
opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
for name, kw, W in [("C3", dict(n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400), 1),
                    ("C4", dict(n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400), 1),
                    ("C4x8", dict(n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400), 8),
                    ("SH80k", dict(n_kf=50, n_pts=80000, n_fixed=5, fixed_obs_per_kf=400), 1)]:
    if os.environ.get("TIME_BA_ONLY") and name not in os.environ["TIME_BA_ONLY"].split(","):
        continue
    wins = [synth.ba_window(seed=4 + i, **kw) for i in range(W)]
    t0 = time.perf_counter(); plan = BAPlan(ctx, wins); t1 = time.perf_counter()
    plan.solve(opt); ctx.sync()
    ts = []
    for _ in range(5):
        a = time.perf_counter(); plan.solve(opt); ctx.sync(); ts.append(time.perf_counter() - a)
    P, X, s = plan.read()
    L = lib(); L.lorb_kernel_timing_enable(ctx.handle, 1)
    plan.solve(opt); ctx.sync()
    res = {}
    for k, nm in [(3, "lin"), (2, "schur"), (4, "chol")]:
        ms, n = C.c_double(0), C.c_int(0)
        L.lorb_kernel_timing_read(ctx.handle, k, C.byref(ms), C.byref(n)); res[nm] = (ms.value / max(n.value, 1), n.value)
    L.lorb_kernel_timing_enable(ctx.handle, 0)
    print("pm", name, "W", W, "plan %.1f ms" % ((t1 - t0) * 1e3), "solve med %.3f ms" % (np.median(ts) * 1e3),
          "it/s %.0f" % (10 * W / np.median(ts)), s[0], "per-kernel ms", res, flush=True)
    plan.close()
