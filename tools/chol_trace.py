"""Diagnostic: per-panel event timeline of k_ba_chol_2s on the C4 window (cycles, s_memtime).
Needs LORB_LIB_PATH=variants/liblorb_trace.so (tools/build_variant.sh trace -DLORB_CHOL_TRACE)."""
import sys, os, ctypes as C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lorb_slam_amd import synth, _abi as A
from lorb_slam_amd.runtime import Context, BAPlan, lib
ctx = Context(0)
opt = A.LMOptions.default(max_num_iterations=1, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
plan = BAPlan(ctx, [synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)])
for _ in range(4):
    plan.solve(opt)
ctx.sync()
out = (C.c_ulonglong * 512)()
lib().lorb_ba_plan_debug_stamps(plan._p, out)
v = list(out)
def chain(base, n):
    return [(v[base + 3 * p], v[base + 3 * p + 1], v[base + 3 * p + 2]) for p in range(n)]
def upd(base, n):
    return [tuple(v[base + 4 * p + k] for k in range(4)) for p in range(n)]
print("top chain  (ready, factored, posted):")
for p, e in enumerate(chain(0, 11)): print("  ", p, e, "factor", e[1] - e[0], "store", e[2] - e[1])
print("top update (Tn loaded, L got, handed, done):")
for p, e in enumerate(upd(64, 11)): print("  ", p, e)
print("bottom chain:")
for p, e in enumerate(chain(128, 8)): print("  ", p, e, "factor", e[1] - e[0], "store", e[2] - e[1])
print("bottom update:")
for p, e in enumerate(upd(160, 8)): print("  ", p, e)
names = ["w2 T done", "w2 got X", "w3 X written", "w0 M start", "w0 M done", "w0 bs start", "w0 bs M done",
         "w0 bs T done", "stage top done", "stage bot done", "linv top done", "linv bot done", "w1 bs B done", "end",
         "w2 combined", "w2 M handed", "K/G top start", "K/G top done", "K/G bot start", "K/G bot done",
         "w1 woke", "w1 init done", "w3 w top start", "w3 w top done", "w1 w bot start", "w1 w bot done",
         "w4 comb start", "w5 comb start", "w6 comb start", "w7 comb start",
         "w4 comb done", "w5 comb done", "w6 comb done", "w7 comb done"]
for k, nm in enumerate(names): print(f"{nm:16s} {v[200 + k]}")
plan.close()
print("entry -> traced t0:", v[252] - v[250], " traced t0 -> epilogue issued (thread 0):", v[251] - v[252])
print("G steps top (wave 5):", [v[320 + i] for i in range(16)])
print("G steps bottom (wave 7):", [v[400 + i] for i in range(16)])
for nm, b in (("top", 320), ("bottom", 400)):
    st = [(v[b + 3 * i], v[b + 3 * i + 1], v[b + 3 * i + 2]) for i in range(24) if v[b + 3 * i]]
    print(f"bs {nm} blocks (start, after publish+wait, after product):", st)
print("linv top (start, end):", [(v[256 + 2 * p], v[257 + 2 * p]) for p in range(8)])
print("linv bot (start, end):", [(v[288 + 2 * p], v[289 + 2 * p]) for p in range(8)])
