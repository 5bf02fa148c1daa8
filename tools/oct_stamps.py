"""Diagnostic: cycle stamps of k_orb_octree's LDS path per level (lorb_orb_debug_octree) on the
tools/time_orb.py image: gather, initial nodes, then per pass (B done, E done, pass done), final."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from lorb_slam_amd import _abi as A, synth  # noqa: E402
from lorb_slam_amd.runtime import Context, lib  # noqa: E402

ctx = Context(0)
img = synth.orb_problem(seed=73, n_kps=1)["pyr"][0]
sf = A.f32(synth.scale_factors())
pyr = ctx.orb_pyramid(img, sf) if hasattr(ctx, "orb_pyramid") else O.orb_pyramid(img, sf)
nd = O.orb_features_per_level(1000)
buf, P = A.pack_pyramid(pyr)
P.data = buf.ctypes.data
tr = np.zeros(8 * (64 * 72 + 16384), np.int32)
for _ in range(3):
    rc = lib().lorb_orb_debug_octree(ctx.handle, C.byref(P), A.ptr(A.i32(nd), C.c_int32), A.ptr(sf, C.c_float), 20, 7,
                                     A.ptr(tr, C.c_int32))
    assert rc == 0
st = tr[8 * 64 * 72:].reshape(8, 16384)[:, :60]
for l in range(8):
    v = st[l][st[l] > 0]
    print(l, "stamps (cycles):", v.tolist(), "deltas:", np.diff(np.concatenate([[0], v])).tolist(), flush=True)
