"""Device time of the SURVEY §8f rows on resident inputs (HIP events around N back-to-back calls of
the _dev entry points) and the single-thread oracle on the same inputs.
  lorb_compute_stereo_matches_dev  (row 2, one stereo frame: 2000 left / 2800 right keypoints, 752x480)
  lorb_track_local_map_dev         (row 1, 2000 keypoints x 3000 local map points)
  lorb_compute_descriptor_dev      (row 4, 3000 points x 8 observations)
  lorb_orb_describe_dev            (row 3 descriptor stage, 2000 keypoints on a 752x480 8-level pyramid)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from lorb_slam_amd import _abi as A, synth  # noqa: E402

from lorb_slam_amd.runtime import Context, lib  # noqa: E402
import lorb_slam_amd.window  # noqa: E402,F401

N = int(os.environ.get("ROWS_N", "200"))
ctx = Context(0)
keep = []


def dev(a, dtype):
    d = ctx.to_device(np.ascontiguousarray(a, dtype))
    keep.append(d)
    return d.ptr


def timed(fn):
    fn(); ctx.sync()
    ctx.timer_mark(0)
    for _ in range(N):
        fn()
    ctx.timer_mark(1)
    ctx.sync()
    return ctx.timer_ms(0, 1) * 1e3 / N


def cpu(fn, reps=5):
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) * 1e6 / reps


out = {}
# row 2: stereo
sp = synth.stereo_problem(seed=21)
fps = A.make_frame_params(sp["fp"])
bl, pl = A.pack_pyramid(sp["pyr_l"]); br, pr = A.pack_pyramid(sp["pyr_r"])
pl.data, pr.data = dev(bl, np.uint8), dev(br, np.uint8)
kl = A.StereoKeys(len(sp["left"]["x"]), *[dev(sp["left"][k], t) for k, t in
                                          (("x", np.float32), ("y", np.float32), ("octave", np.int32), ("desc", np.uint8))])
kr = A.StereoKeys(len(sp["right"]["x"]), *[dev(sp["right"][k], t) for k, t in
                                           (("x", np.float32), ("y", np.float32), ("octave", np.int32), ("desc", np.uint8))])
ur, dp = ctx.empty(kl.n, np.float32), ctx.empty(kl.n, np.float32)
us = timed(lambda: ctx.check(lib().lorb_compute_stereo_matches_dev(ctx.handle, C.byref(fps), C.byref(kl), C.byref(kr),
                                                                   C.byref(pl), C.byref(pr), ur.ptr, dp.ptr), "stereo"))
o = O.compute_stereo_matches(sp["fp"], sp["left"], sp["right"], sp["pyr_l"], sp["pyr_r"])
assert np.array_equal(ur.numpy(), o[0])
out["stereo"] = dict(gpu_us=us, cpu_us=cpu(lambda: O.compute_stereo_matches(sp["fp"], sp["left"], sp["right"],
                                                                           sp["pyr_l"], sp["pyr_r"])),
                     n_left=kl.n, n_right=kr.n, n_depth=int((o[0] >= 0).sum()))
# row 1: local-map tracking
lp = synth.local_map_problem(seed=11)
fps1 = A.make_frame_params(lp["fp"])
k = lp["kps"]; m = lp["pts"]
K = A.KeypointsDev(len(k["x"]), dev(k["x"], np.float32), dev(k["y"], np.float32), dev(k["octave"], np.int32),
                   dev(k["angle"], np.float32), dev(k["u_right"], np.float32), dev(k["desc"], np.uint8))
M = A.MapPointsDev(len(m["max_dist"]), dev(m["pos"], np.float32), dev(m["normal"], np.float32),
                   dev(m["max_dist"], np.float32), dev(m["min_dist"], np.float32), dev(m["desc"], np.uint8),
                   dev(m["locked"], np.uint8), dev(m["is_bad"], np.uint8), dev(m["in_frame"], np.uint8))
ss = dev(lp["slot_state"], np.uint8)
npt, nk = M.n, K.n
iv, tr, lv = ctx.empty(npt, np.uint8), ctx.empty((4, npt), np.float32), ctx.empty(npt, np.int32)
asg, nm = ctx.empty(nk, np.int32), ctx.empty(1, np.int32)
T = A.f32(lp["Tcw"]).reshape(16)
us = timed(lambda: ctx.check(lib().lorb_track_local_map_dev(ctx.handle, C.byref(fps1), A.ptr(T, C.c_float), C.byref(K), ss,
                                                            C.byref(M), C.c_float(0.5), C.c_float(1.0), iv.ptr, tr.ptr,
                                                            lv.ptr, asg.ptr, nm.ptr), "track"))
fr, a, n = O.track_local_map(lp["fp"], lp["Tcw"], k, lp["slot_state"], m)
assert np.array_equal(asg.numpy(), a) and int(nm.numpy()[0]) == n
out["track_local_map"] = dict(gpu_us=us, cpu_us=cpu(lambda: O.track_local_map(lp["fp"], lp["Tcw"], k, lp["slot_state"], m)),
                              n_kps=nk, n_points=npt, n_matches=n)
# row 4: ComputeDescriptor
rng = np.random.default_rng(3)
npd, nobs = 3000, 8
d_off = np.arange(0, (npd + 1) * nobs, nobs, dtype=np.int32)
desc = rng.integers(0, 256, size=(npd * nobs, 32), dtype=np.uint8)
dd, doff = dev(desc, np.uint8), dev(d_off, np.int32)
best, outd = ctx.empty(npd, np.int32), ctx.empty((npd, 32), np.uint8)
us = timed(lambda: ctx.check(lib().lorb_compute_descriptor_dev(ctx.handle, C.c_int32(npd), doff, dd, best.ptr, outd.ptr),
                             "compute_descriptor"))
out["compute_descriptor"] = dict(gpu_us=us, cpu_us=cpu(lambda: O.compute_descriptor(d_off, desc)), n_points=npd,
                                 obs_per_point=nobs)
# row 3: ORB descriptor stage (blur of all 8 levels + orientation + rBRIEF)
op = synth.orb_problem(seed=31, n_kps=2000)
buf, P = A.pack_pyramid(op["pyr"])
P.data = dev(buf, np.uint8)
ox, oy, ol, opat = (dev(op[k], t) for k, t in (("x", np.float32), ("y", np.float32), ("level", np.int32),
                                               ("pattern", np.int32)))
oang, odesc = ctx.empty(2000, np.float32), ctx.empty((2000, 32), np.uint8)
us = timed(lambda: ctx.check(lib().lorb_orb_describe_dev(ctx.handle, C.byref(P), C.c_int32(2000), ox, oy, ol, opat,
                                                         oang.ptr, odesc.ptr), "orb_describe"))
ra, rd = O.orb_describe(op["pyr"], op["x"], op["y"], op["level"], op["pattern"])
assert np.array_equal(odesc.numpy(), rd) and np.array_equal(oang.numpy(), ra)
out["orb_describe"] = dict(gpu_us=us, cpu_us=cpu(lambda: O.orb_describe(op["pyr"], op["x"], op["y"], op["level"],
                                                                        op["pattern"])),
                           n_kps=2000, pyramid="752x480, 8 levels x 1.2")
# row 3: the whole extractor on one 752x480 image: pyramid + FAST cells + retention (host) + describe
img = synth.orb_problem(seed=73, n_kps=1)["pyr"][0]
sf = synth.scale_factors()
nd = O.orb_features_per_level(1000)
pat = np.random.default_rng(9).integers(-13, 13, size=1024).astype(np.int32)


def extract_gpu():
    p = ctx.orb_pyramid(img, sf)
    d = ctx.orb_detect(p, nd, sf)
    return ctx.orb_describe(p, d["x"], d["y"], d["octave"], pat)


def extract_cpu():
    p = O.orb_pyramid(img, sf)
    d = O.orb_detect(p, nd, sf)
    return O.orb_describe(p, d["x"], d["y"], d["octave"], pat)


def wall(fn, reps):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) * 1e6 / reps


out["orb_extract"] = dict(gpu_us=wall(extract_gpu, 20), cpu_us=wall(extract_cpu, 3),
                          note="host API calls incl. H2D/D2H per stage (not device-resident)")
print(json.dumps(out))
