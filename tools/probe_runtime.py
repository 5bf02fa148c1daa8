"""GPU-box probe: does liblorb.so work with and without torch loaded first?"""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
if len(sys.argv) > 1 and sys.argv[1] == "torch_first":
    import torch
    print("torch", torch.__version__, "hip", torch.version.hip)
import numpy as np
import oracle as O
from lorb_slam_amd import synth
from lorb_slam_amd.runtime import Context, device_count
print("devices", device_count())
ctx = Context(0)
q, t, lev = synth.bf_problem(seed=2, nq=300, nt=400, n_planted=100, random_levels=True)
got, _ = ctx.bf_top2([q], [t], [lev])
ref = O.bf_top2(q, t, lev)
print("top2 ok", all(np.array_equal(got[k], ref[k]) for k in ref))
maps = open("/proc/self/maps").read()
print("hip libs:", sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l}))
