"""Diagnostics: the LM solve of 8 independent C4 windows split into K plans of 8 / K windows, one
context (stream) per plan, the K solves enqueued back to back from one host thread (the solve is
stream-ordered), so that one plan's Cholesky (one CU per window) can run beside another plan's
point-group kernels.  Prints ms per 8-window solve for each K."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import synth  # noqa: E402
from lorb_slam_amd.runtime import BAPlan, Context  # noqa: E402

ctx0 = Context(0)
wins = [synth.ba_window(seed=40 + i, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400) for i in range(8)]
opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                          parameter_tolerance=0.0)
ks = [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]
extra = [Context(0) for _ in range(max(ks) - 1)]
ctxs = [ctx0] + extra
for K in ks:
    per = 8 // K
    plans = [BAPlan(ctxs[k], wins[k * per:(k + 1) * per]) for k in range(K)]
    for _ in range(2):
        for p in plans:
            p.solve(opt)
    for c in ctxs[:K]:
        c.sync()
    res = []
    for rep in range(3):
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            for p in plans:
                p.solve(opt)
        for c in ctxs[:K]:
            c.sync()
        res.append((time.perf_counter() - t0) / n * 1e3)
    costs = [s["final_cost"] for p in plans for s in p.read()[2]]
    print("K=%d plans x %d windows: ms per 8-window solve %s -> %.0f LM it/s; cost w0 %.9e" %
          (K, per, " ".join("%.3f" % r for r in res), 80.0 / (min(res) / 1e3), costs[0]), flush=True)
    for p in plans:
        p.close()
