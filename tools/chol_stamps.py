"""Diagnostic: Cholesky phase cycles (s_memtime) for the C4 window; needs LORB_LIB_PATH=stamps build."""
import sys, os, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lorb_slam_amd import synth, _abi as A
from lorb_slam_amd.runtime import Context, BAPlan, lib
ctx = Context(0)
opt = A.LMOptions.default(max_num_iterations=1, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
for kw in [dict(n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400), dict(n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)]:
    plan = BAPlan(ctx, [synth.ba_window(seed=4, **kw)])
    for _ in range(3):
        plan.solve(opt)
    ctx.sync()
    out = (C.c_ulonglong * 8)()
    lib().lorb_ba_plan_debug_stamps(plan._p, out)
    print(kw["n_kf"], "stamps", list(out[:8]))
    plan.close()
