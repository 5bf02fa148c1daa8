"""Diagnostics: per-phase cycles of k_ba_ls (point-major linearisation + Schur partials) from a
LORB_LS_STAMPS build (tools/build_variant.sh lsst -DLORB_LS_STAMPS; run with
LORB_LIB_PATH=variants/liblorb_lsst.so).  One eager solve per window shape; the stamps are the last
iteration's.  Prints the median / p90 cycles of phases A (linearisation), B (points), C (slots),
D (block rows), E (partials' reduction), the spread of the groups' start times, and the kernel span."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lorb_slam_amd import _abi as A, synth  # noqa: E402
from lorb_slam_amd.runtime import BAPlan, Context, lib  # noqa: E402

ctx = Context(0)
L = lib()
opt = A.LMOptions.default(max_num_iterations=2, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
for name, kw in [("C4", dict(n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)),
                 ("SH80k", dict(n_kf=50, n_pts=80000, n_fixed=5, fixed_obs_per_kf=400))]:
    plan = BAPlan(ctx, [synth.ba_window(seed=4, **kw)])
    L.lorb_kernel_timing_enable(ctx.handle, 1)  # eager launches
    plan.solve(opt)
    ctx.sync()
    L.lorb_kernel_timing_enable(ctx.handle, 0)
    info = plan.info() if hasattr(plan, "info") else {}
    ng = int(info.get("point_groups", 0)) or 4096
    buf = (C.c_ulonglong * (8 * max(ng, 1)))()
    ctx.check(L.lorb_ba_plan_debug_stamps(plan._p, buf), "stamps")
    st = np.frombuffer(buf, np.uint64).reshape(-1, 8).astype(np.int64)
    st = st[st[:, 0] > 0]
    ph = np.diff(st[:, :6], axis=1)
    t0 = st[:, 0] - st[:, 0].min()
    print(name, "groups", len(st), "kernel span %.0f cycles" % (st[:, 5].max() - st[:, 0].min()),
          "start spread p50 %.0f p90 %.0f" % (np.median(t0), np.percentile(t0, 90)), flush=True)
    for i, nm in enumerate("ABCDE"):
        print("  %s median %7.0f p90 %7.0f max %7.0f" % (nm, np.median(ph[:, i]), np.percentile(ph[:, i], 90), ph[:, i].max()))
    plan.close()
