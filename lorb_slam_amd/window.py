"""ctypes bindings of the windowed matchers and frame callees (a4, a5, a8, a20) of liblorb.so."""
import ctypes as C

import numpy as np

from . import _abi as A
from .runtime import Context, lib


def _search_by_projection_frame(self, fp, cur_Tcw, cur_kps, cur_slot_state, last, th):
    keep = A.KeepAlive()
    fps = A.make_frame_params(fp)
    k = A.make_keypoints(cur_kps, keep)
    lf = A.make_last_frame(last, keep)
    T = keep.keep(A.f32(cur_Tcw).reshape(16))
    ss = keep.keep(A.u8(cur_slot_state)) if cur_slot_state is not None else None
    assign = np.empty(max(1, k.n), np.int32)
    nm = C.c_int32(0)
    self.check(lib().lorb_search_by_projection_frame(
        self.handle, C.byref(fps), A.ptr(T, C.c_float), C.byref(k), A.ptr(ss, C.c_uint8), C.byref(lf),
        C.c_float(th), A.ptr(assign, C.c_int32), C.byref(nm)), "lorb_search_by_projection_frame")
    return assign[: k.n].copy(), nm.value


def _search_by_projection_local(self, fp, kps, slot_state, pts, th):
    keep = A.KeepAlive()
    fps = A.make_frame_params(fp)
    k = A.make_keypoints(kps, keep)
    lp = A.make_local_points(pts, keep)
    ss = keep.keep(A.u8(slot_state)) if slot_state is not None else None
    assign = np.empty(max(1, k.n), np.int32)
    nm = C.c_int32(0)
    self.check(lib().lorb_search_by_projection_local(
        self.handle, C.byref(fps), C.byref(k), A.ptr(ss, C.c_uint8), C.byref(lp), C.c_float(th),
        A.ptr(assign, C.c_int32), C.byref(nm)), "lorb_search_by_projection_local")
    return assign[: k.n].copy(), nm.value


def _is_in_frustum(self, fp, Tcw, fpts, cos_limit=0.5):
    keep = A.KeepAlive()
    fps = A.make_frame_params(fp)
    p = A.make_frustum_points(fpts, keep)
    T = keep.keep(A.f32(Tcw).reshape(16))
    n = p.n
    out = dict(in_view=np.zeros(max(n, 1), np.uint8), proj_x=np.zeros(max(n, 1), np.float32),
               proj_y=np.zeros(max(n, 1), np.float32), proj_xr=np.zeros(max(n, 1), np.float32),
               pred_level=np.zeros(max(n, 1), np.int32), view_cos=np.zeros(max(n, 1), np.float32))
    self.check(lib().lorb_is_in_frustum(
        self.handle, C.byref(fps), A.ptr(T, C.c_float), C.byref(p), C.c_float(cos_limit),
        A.ptr(out["in_view"], C.c_uint8), A.ptr(out["proj_x"], C.c_float), A.ptr(out["proj_y"], C.c_float),
        A.ptr(out["proj_xr"], C.c_float), A.ptr(out["pred_level"], C.c_int32),
        A.ptr(out["view_cos"], C.c_float)), "lorb_is_in_frustum")
    return {k_: v[:n] for k_, v in out.items()}


def _unproject_stereo(self, fp, Tcw, x, y, depth):
    fps = A.make_frame_params(fp)
    T = A.f32(Tcw).reshape(16)
    x = A.f32(x); y = A.f32(y); d = A.f32(depth)
    out = np.zeros((max(len(x), 1), 3), np.float32)
    self.check(lib().lorb_unproject_stereo(self.handle, C.byref(fps), A.ptr(T, C.c_float), C.c_int32(len(x)),
                                           A.ptr(x, C.c_float), A.ptr(y, C.c_float), A.ptr(d, C.c_float),
                                           A.ptr(out, C.c_float)), "lorb_unproject_stereo")
    return out[: len(x)]


def _track_local_map(self, fp, Tcw, kps, slot_state, pts, cos_limit=0.5, th=1.0):
    """lorb_track_local_map_dev on device copies of the inputs (they stay resident for the call)."""
    keep = []

    def dev(a, dtype):
        d = self.to_device(np.ascontiguousarray(a, dtype))
        keep.append(d)
        return d.ptr

    nk, npt = len(kps["x"]), len(pts["max_dist"])
    k = A.KeypointsDev(nk, dev(kps["x"], np.float32), dev(kps["y"], np.float32), dev(kps["octave"], np.int32),
                       dev(kps["angle"], np.float32),
                       dev(kps["u_right"], np.float32) if kps.get("u_right") is not None else None,
                       dev(kps["desc"], np.uint8))
    m = A.MapPointsDev(npt, dev(pts["pos"], np.float32), dev(pts["normal"], np.float32), dev(pts["max_dist"], np.float32),
                       dev(pts["min_dist"], np.float32), dev(pts["desc"], np.uint8), dev(pts["locked"], np.uint8),
                       dev(pts["is_bad"], np.uint8) if pts.get("is_bad") is not None else None,
                       dev(pts["in_frame"], np.uint8) if pts.get("in_frame") is not None else None)
    ss = dev(slot_state, np.uint8) if slot_state is not None else None
    iv, tr, lv = self.empty(max(npt, 1), np.uint8), self.empty((4, max(npt, 1)), np.float32), self.empty(max(npt, 1), np.int32)
    asg, nm = self.empty(max(nk, 1), np.int32), self.empty(1, np.int32)
    fps = A.make_frame_params(fp)
    T = A.f32(Tcw).reshape(16)
    self.check(lib().lorb_track_local_map_dev(self._p, C.byref(fps), A.ptr(T, C.c_float), C.byref(k), ss, C.byref(m),
                                              C.c_float(cos_limit), C.c_float(th), iv.ptr, tr.ptr, lv.ptr, asg.ptr, nm.ptr),
               "lorb_track_local_map_dev")
    trk = tr.numpy().reshape(4, -1)[:, :npt] if npt else np.zeros((4, 0), np.float32)
    out = dict(in_view=iv.numpy()[:npt], proj_x=trk[0], proj_y=trk[1], proj_xr=trk[2], view_cos=trk[3],
               pred_level=lv.numpy()[:npt], assign=asg.numpy()[:nk], nmatches=int(nm.numpy()[0]))
    for a in keep + [iv, tr, lv, asg, nm]:
        a.free()
    return out


def _compute_stereo_matches(self, fp, left, right, pyr_l, pyr_r, device_resident=False):
    """Frame::ComputeStereoMatches -> (u_right, depth).  device_resident=True stages every input in
    device memory first and calls lorb_compute_stereo_matches_dev (the async form)."""
    fps = A.make_frame_params(fp)
    n = len(left["x"])
    bl, pl = A.pack_pyramid(pyr_l)
    br, pr = A.pack_pyramid(pyr_r)
    if not device_resident:
        keep = A.KeepAlive()
        kl, kr = A.make_stereo_keys(left, keep), A.make_stereo_keys(right, keep)
        pl.data, pr.data = bl.ctypes.data, br.ctypes.data
        ur, dp = np.empty(max(n, 1), np.float32), np.empty(max(n, 1), np.float32)
        self.check(lib().lorb_compute_stereo_matches(self._p, C.byref(fps), C.byref(kl), C.byref(kr), C.byref(pl),
                                                     C.byref(pr), A.ptr(ur, C.c_float), A.ptr(dp, C.c_float)),
                   "lorb_compute_stereo_matches")
        return ur[:n].copy(), dp[:n].copy()
    keep = []

    def dev(a, dtype):
        d = self.to_device(np.ascontiguousarray(a, dtype))
        keep.append(d)
        return d.ptr

    def keys(k):
        return A.StereoKeys(len(k["x"]), dev(k["x"], np.float32), dev(k["y"], np.float32), dev(k["octave"], np.int32),
                            dev(k["desc"], np.uint8))

    kl, kr = keys(left), keys(right)
    pl.data, pr.data = dev(bl, np.uint8), dev(br, np.uint8)
    ur, dp = self.empty(max(n, 1), np.float32), self.empty(max(n, 1), np.float32)
    keep += [ur, dp]
    self.check(lib().lorb_compute_stereo_matches_dev(self._p, C.byref(fps), C.byref(kl), C.byref(kr), C.byref(pl),
                                                     C.byref(pr), ur.ptr, dp.ptr), "lorb_compute_stereo_matches_dev")
    out = ur.numpy()[:n], dp.numpy()[:n]
    for a in keep:
        a.free()
    return out


def _orb_describe(self, pyr, x, y, level, pattern, device_resident=False):
    """ORBextractor descriptor stage -> (angle, desc).  device_resident=True stages the inputs in
    device memory first and calls lorb_orb_describe_dev."""
    buf, P = A.pack_pyramid(pyr)
    x, y, level, pattern = A.f32(x), A.f32(y), A.i32(level), A.i32(pattern).reshape(-1)
    n = len(x)
    if not device_resident:
        P.data = buf.ctypes.data
        ang = np.empty(max(n, 1), np.float32)
        desc = np.empty((max(n, 1), 32), np.uint8)
        self.check(lib().lorb_orb_describe(self._p, C.byref(P), C.c_int32(n), A.ptr(x, C.c_float), A.ptr(y, C.c_float),
                                           A.ptr(level, C.c_int32), A.ptr(pattern, C.c_int32), A.ptr(ang, C.c_float),
                                           A.ptr(desc, C.c_uint8)), "lorb_orb_describe")
        return ang[:n].copy(), desc[:n].copy()
    keep = [self.to_device(a) for a in (buf, x, y, level, pattern)]
    P.data = keep[0].ptr
    ang, desc = self.empty(max(n, 1), np.float32), self.empty((max(n, 1), 32), np.uint8)
    keep += [ang, desc]
    self.check(lib().lorb_orb_describe_dev(self._p, C.byref(P), C.c_int32(n), keep[1].ptr, keep[2].ptr, keep[3].ptr,
                                           keep[4].ptr, ang.ptr, desc.ptr), "lorb_orb_describe_dev")
    out = ang.numpy()[:n], desc.numpy()[:n]
    for a in keep:
        a.free()
    return out


def _orb_fast_cells(self, pyr, ini_th=20, min_th=7, max_kp=200000, max_cells=4096):
    """FAST stage of ORBextractor::ComputeKeyPointsOctTree (src/ORBextractor.cpp:803-872): per-cell
    FAST with the empty-cell fallback.  Returns x, y, response (level coordinates) and the
    cell_base / cell_off tables."""
    buf, P = A.pack_pyramid(pyr)
    P.data = buf.ctypes.data
    x, y, r = np.zeros(max_kp, np.float32), np.zeros(max_kp, np.float32), np.zeros(max_kp, np.float32)
    base = np.zeros(len(pyr) + 1, np.int32)
    off = np.zeros(max_cells + len(pyr) + 1, np.int32)
    n = C.c_int32(0)
    self.check(lib().lorb_orb_fast_cells(self._p, C.byref(P), C.c_int32(ini_th), C.c_int32(min_th),
                                         C.c_int32(max_kp), A.ptr(x, C.c_float), A.ptr(y, C.c_float),
                                         A.ptr(r, C.c_float), C.c_int32(max_cells), A.ptr(base, C.c_int32),
                                         A.ptr(off, C.c_int32), C.byref(n)), "lorb_orb_fast_cells")
    k = n.value
    return dict(x=x[:k].copy(), y=y[:k].copy(), response=r[:k].copy(), cell_base=base,
                cell_off=off[:base[-1] + len(pyr)].copy())


def _orb_detect(self, pyr, n_desired, scale_factors, ini_th=20, min_th=7, max_kp=100000):
    """ComputeKeyPointsOctTree without orientation (src/ORBextractor.cpp:799-892): FAST cells and
    DistributeOctTree on the device."""
    buf, P = A.pack_pyramid(pyr)
    P.data = buf.ctypes.data
    nd, sf = A.i32(n_desired), A.f32(scale_factors)
    x, y, sz, r = (np.zeros(max_kp, np.float32) for _ in range(4))
    o = np.zeros(max_kp, np.int32)
    lo = np.zeros(len(pyr) + 1, np.int32)
    n = C.c_int32(0)
    self.check(lib().lorb_orb_detect(self._p, C.byref(P), A.ptr(nd, C.c_int32), A.ptr(sf, C.c_float), C.c_int32(ini_th),
                                     C.c_int32(min_th), C.c_int32(max_kp), A.ptr(x, C.c_float), A.ptr(y, C.c_float),
                                     A.ptr(o, C.c_int32), A.ptr(sz, C.c_float), A.ptr(r, C.c_float),
                                     A.ptr(lo, C.c_int32), C.byref(n)), "lorb_orb_detect")
    k = n.value
    return dict(x=x[:k].copy(), y=y[:k].copy(), octave=o[:k].copy(), size=sz[:k].copy(), response=r[:k].copy(),
                level_off=lo)


def _orb_extract(self, img, n_desired, scale_factors, pattern, ini_th=20, min_th=7, max_kp=100000):
    """The whole ORBextractor::operator() (src/ORBextractor.cpp:1087-1151) on the device."""
    img = A.u8(img)
    nd, sf, pat = A.i32(n_desired), A.f32(scale_factors), A.i32(pattern).reshape(-1)
    x, y, sz, ang, r = (np.zeros(max_kp, np.float32) for _ in range(5))
    o = np.zeros(max_kp, np.int32)
    desc = np.zeros((max_kp, 32), np.uint8)
    lo = np.zeros(len(sf) + 1, np.int32)
    n = C.c_int32(0)
    self.check(lib().lorb_orb_extract(self._p, A.ptr(img, C.c_uint8), C.c_int32(img.shape[0]), C.c_int32(img.shape[1]),
                                      C.c_int32(img.shape[1]), C.c_int32(len(sf)), A.ptr(sf, C.c_float),
                                      A.ptr(nd, C.c_int32), C.c_int32(ini_th), C.c_int32(min_th), A.ptr(pat, C.c_int32),
                                      C.c_int32(max_kp), A.ptr(x, C.c_float), A.ptr(y, C.c_float), A.ptr(o, C.c_int32),
                                      A.ptr(sz, C.c_float), A.ptr(ang, C.c_float), A.ptr(r, C.c_float),
                                      A.ptr(desc, C.c_uint8), A.ptr(lo, C.c_int32), C.byref(n)), "lorb_orb_extract")
    k = n.value
    return dict(x=x[:k].copy(), y=y[:k].copy(), octave=o[:k].copy(), size=sz[:k].copy(), angle=ang[:k].copy(),
                response=r[:k].copy(), desc=desc[:k].copy(), level_off=lo)


def _orb_pyramid(self, img, scale_factors):
    """ORBextractor::ComputePyramid on the device -> list of level images."""
    img = A.u8(img)
    sf = A.f32(scale_factors)
    total = int(sum(int(np.rint(np.float32(img.shape[0]) * (np.float32(1) / s))) *
                    int(np.rint(np.float32(img.shape[1]) * (np.float32(1) / s))) for s in sf))
    out = np.zeros(total + 16, np.uint8)
    P = A.ImagePyramid()
    self.check(lib().lorb_orb_pyramid(self._p, A.ptr(img, C.c_uint8), C.c_int32(img.shape[0]), C.c_int32(img.shape[1]),
                                      C.c_int32(img.shape[1]), C.c_int32(len(sf)), A.ptr(sf, C.c_float),
                                      A.ptr(out, C.c_uint8), C.c_int64(len(out)), C.byref(P)), "lorb_orb_pyramid")
    return [out[P.offset[l]:P.offset[l] + P.rows[l] * P.cols[l]].reshape(P.rows[l], P.cols[l]).copy()
            for l in range(len(sf))]


Context.orb_pyramid = _orb_pyramid
Context.orb_extract = _orb_extract
Context.orb_detect = _orb_detect
Context.orb_fast_cells = _orb_fast_cells
Context.orb_describe = _orb_describe
Context.compute_stereo_matches = _compute_stereo_matches
Context.track_local_map = _track_local_map
Context.search_by_projection_frame = _search_by_projection_frame
Context.search_by_projection_local = _search_by_projection_local
Context.is_in_frustum = _is_in_frustum
Context.unproject_stereo = _unproject_stereo
