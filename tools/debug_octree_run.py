"""Diagnostic: k_orb_octree's per-pass trace (lorb_orb_debug_octree) against the pure-Python
DistributeOctTree of tools/debug_octree.py, every level, on synth.orb_problem(seed) (default 61)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import debug_octree as D  # noqa: E402
import oracle as O  # noqa: E402
from lorb_slam_amd import _abi as A, synth  # noqa: E402
from lorb_slam_amd.runtime import Context, lib  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 61
nfeat = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
ctx = Context(0)
pyr = synth.orb_problem(seed=seed, n_kps=1)["pyr"]
nd = O.orb_features_per_level(nfeat)
buf, P = A.pack_pyramid(pyr)
P.data = buf.ctypes.data
tr = np.zeros(8 * (64 * 72 + 16384), np.int32)
sf = A.f32(synth.scale_factors())
rc = lib().lorb_orb_debug_octree(ctx.handle, C.byref(P), A.ptr(A.i32(nd), C.c_int32), A.ptr(sf, C.c_float), 20, 7,
                                 A.ptr(tr, C.c_int32))
assert rc == 0
gp = tr[8 * 64 * 72:].reshape(8, 16384)
tr = tr[:8 * 64 * 72].reshape(8, 64, 72)
f = O.orb_fast_cells(pyr)
for l, p in enumerate(pyr):
    b0, b1 = f["cell_off"][f["cell_base"][l] + l], f["cell_off"][f["cell_base"][l + 1] + l]
    kx, ky, kr = f["x"][b0:b1] - 16, f["y"][b0:b1] - 16, f["response"][b0:b1]
    t = []
    perms = []
    D.sim(kx, ky, kr, 16, p.shape[1] - 16, 16, p.shape[0] - 16, nd[l], t, perms)
    g0 = gp[l, 64:64 + len(kx)]
    d = np.flatnonzero(g0 != np.asarray(perms[0]))
    print("level", l, "pass-0 positions differing:", len(d), d[:10].tolist(), g0[d[:5]].tolist(), np.asarray(perms[0])[d[:5]].tolist())
    bad = 0
    for k, row in enumerate(t):
        g = tr[l, k][:len(row)].tolist()
        if row != g:
            bad += 1
            if bad <= 2:
                print(l, k, "sim", row, "\n       gpu", g, flush=True)
    print("level", l, "keys", len(kx), "passes", len(t), "mismatching passes", bad, flush=True)
