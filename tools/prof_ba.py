"""Profile helper: C4 window BA, 10 LM iterations, a few solves (for rocprofv3)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lorb_slam_amd import synth, _abi as A
from lorb_slam_amd.runtime import Context, BAPlan
W = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ctx = Context(0)
opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
wins = [synth.ba_window(seed=4 + i, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400) for i in range(W)]
plan = BAPlan(ctx, wins)
for _ in range(3):
    plan.solve(opt)
ctx.sync()
print(plan.read()[2][0])
