"""Device time of the whole ORB extraction (ORBextractor::operator(),
src/ORBextractor.cpp:1087-1151) through lorb_orb_extract_dev on a resident 752x480 image: N
back-to-back frames between HIP events on the ctx stream, the per-frame wall time of the same calls
with a stream sync after each frame, and the host-API lorb_orb_extract (H2D + D2H per call) for
comparison.  Run under rocprofv3 --kernel-trace --stats for the per-kernel split
(k_orb_resize / k_orb_fast / k_orb_octree / k_orb_blur / k_orb_desc).
usage: python tools/time_orb.py [--frames N] [--features 1000]"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--features", type=int, default=1000)
    args = ap.parse_args()
    ctx = Context(0)
    img = np.ascontiguousarray(synth.orb_problem(seed=73, n_kps=1)["pyr"][0], np.uint8)
    rows, cols = img.shape
    sf = A.f32(synth.scale_factors())
    nd = A.i32(O.orb_features_per_level(args.features))
    pat = np.random.default_rng(9).integers(-13, 13, size=1024).astype(np.int32)
    L = len(sf)
    cap, pyb = C.c_int32(0), C.c_int64(0)
    ctx.check(lib().lorb_orb_extract_capacity(C.c_int32(rows), C.c_int32(cols), C.c_int32(L), A.ptr(sf, C.c_float),
                                               A.ptr(nd, C.c_int32), C.byref(cap), C.byref(pyb)), "capacity")
    K = cap.value
    d_img, d_pat = ctx.to_device(img), ctx.to_device(pat)
    d_pyr = ctx.empty((pyb.value,), np.uint8)
    outs = [ctx.empty((K,), t) for t in (np.float32, np.float32, np.int32, np.float32, np.float32, np.float32)]
    d_desc = ctx.empty((K, 32), np.uint8)
    d_lo = ctx.empty((L + 1,), np.int32)
    d_n = ctx.empty((1,), np.int32)

    def frame():
        ctx.check(lib().lorb_orb_extract_dev(
            ctx.handle, d_img.as_ptr(C.c_uint8), C.c_int32(rows), C.c_int32(cols), C.c_int32(cols), C.c_int32(L),
            A.ptr(sf, C.c_float), A.ptr(nd, C.c_int32), C.c_int32(20), C.c_int32(7), d_pat.as_ptr(C.c_int32),
            C.c_int32(K), d_pyr.as_ptr(C.c_uint8), C.c_int64(pyb.value), outs[0].as_ptr(C.c_float),
            outs[1].as_ptr(C.c_float), outs[2].as_ptr(C.c_int32), outs[3].as_ptr(C.c_float),
            outs[4].as_ptr(C.c_float), outs[5].as_ptr(C.c_float), d_desc.as_ptr(C.c_uint8),
            d_lo.as_ptr(C.c_int32), d_n.as_ptr(C.c_int32)), "lorb_orb_extract_dev")

    # parity of the resident path against the host API (same kernels) on this image
    frame()
    ctx.sync()
    n = int(d_n.numpy()[0])
    ref = ctx.orb_extract(img, nd, sf, pat)
    ok = n == len(ref["x"]) and np.array_equal(d_desc.numpy()[:n], ref["desc"]) and \
        np.array_equal(outs[0].numpy()[:n], ref["x"])
    for _ in range(3):
        frame()
    ctx.sync()
    ctx.timer_mark(0)
    for _ in range(args.frames):
        frame()
    ctx.timer_mark(1)
    ctx.sync()
    ev_us = ctx.timer_ms(0, 1) * 1e3 / args.frames
    t = time.perf_counter()
    for _ in range(args.frames):
        frame()
        ctx.sync()
    wall_us = (time.perf_counter() - t) * 1e6 / args.frames
    t = time.perf_counter()
    for _ in range(20):
        ctx.orb_extract(img, nd, sf, pat)
    host_us = (time.perf_counter() - t) * 1e6 / 20
    print(json.dumps({"workload": f"orb_extract 752x480, {args.features} features, 8 levels x 1.2",
                      "keypoints": n, "matches_host_api": bool(ok), "frames": args.frames,
                      "stream_us_per_frame": ev_us, "wall_us_per_frame_synced": wall_us,
                      "host_api_us_per_frame": host_us}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
