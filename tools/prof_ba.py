"""Run the C4 local-BA plan (10 LM iterations, tolerances 0) a few times -- a short program for
rocprofv3 --pmc passes on the BA kernels."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lorb_slam_amd import _abi as A, synth  # noqa: E402
from lorb_slam_amd.runtime import BAPlan, Context  # noqa: E402

ctx = Context(0)
opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
plan = BAPlan(ctx, [synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)])
for _ in range(3):
    plan.solve(opt)
ctx.sync()
plan.close()
print("ok")
