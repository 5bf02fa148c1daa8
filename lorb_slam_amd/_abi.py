"""ctypes mirror of include/lorb_c.h (POD structs + prototypes).

Pure plumbing: the compute lives in liblorb.so (HIP, gfx950).  The same struct classes are
used by the test oracle wrapper (oracle/oracle.py), which binds the identical C signatures
of the CPU restatement.
"""
import ctypes as C

import numpy as np

LORB_OK = 0
LORB_TH_HIGH = 100
LORB_TH_LOW = 50
LORB_HISTO_LENGTH = 30
LORB_GRID_ROWS = 48
LORB_GRID_COLS = 64
LORB_MAX_LEVELS = 16
LORB_ASSIGN_UNCHANGED = -1
LORB_ASSIGN_NULL = -2
LORB_SLOT_EMPTY, LORB_SLOT_FREE, LORB_SLOT_LOCKED = 0, 1, 2
TERM_NAMES = {0: "NO_CONVERGENCE", 1: "FUNCTION_TOLERANCE", 2: "GRADIENT_TOLERANCE",
              3: "PARAMETER_TOLERANCE", 4: "MIN_TRUST_REGION_RADIUS", 5: "FAILURE"}

f32p = C.POINTER(C.c_float)
f64p = C.POINTER(C.c_double)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)


class FrameParams(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("b", C.c_float),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float),
                ("n_levels", C.c_int32), ("log_scale_factor", C.c_float),
                ("scale_factors", C.c_float * LORB_MAX_LEVELS)]


class Keypoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("x", f32p), ("y", f32p), ("octave", i32p), ("angle", f32p),
                ("u_right", f32p), ("desc", u8p)]


class LastFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("Tcw", f32p), ("has_mp", u8p), ("outlier", u8p),
                ("mp_locked", u8p), ("mp_pos", f32p), ("mp_desc", u8p), ("octave", i32p),
                ("angle", f32p)]


class LocalPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("track_in_view", u8p), ("is_bad", u8p), ("locked", u8p),
                ("proj_x", f32p), ("proj_y", f32p), ("proj_xr", f32p), ("pred_level", i32p),
                ("view_cos", f32p), ("desc", u8p)]


class FrustumPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("pos", f32p), ("normal", f32p), ("max_dist", f32p),
                ("min_dist", f32p)]


class ImagePyramid(C.Structure):
    _fields_ = [("n_levels", C.c_int32), ("data", C.c_void_p), ("offset", C.c_int64 * LORB_MAX_LEVELS),
                ("rows", C.c_int32 * LORB_MAX_LEVELS), ("cols", C.c_int32 * LORB_MAX_LEVELS),
                ("step", C.c_int32 * LORB_MAX_LEVELS)]


class StereoKeys(C.Structure):
    _fields_ = [("n", C.c_int32), ("x", C.c_void_p), ("y", C.c_void_p), ("octave", C.c_void_p), ("desc", C.c_void_p)]


def pack_pyramid(levels):
    """list of 2-D uint8 images -> (one contiguous byte buffer, ImagePyramid with data=None)."""
    p = ImagePyramid()
    p.n_levels = len(levels)
    off = 0
    for l, im in enumerate(levels):
        p.offset[l], p.rows[l], p.cols[l], p.step[l] = off, im.shape[0], im.shape[1], im.shape[1]
        off += im.size
    buf = np.concatenate([np.ascontiguousarray(im, np.uint8).reshape(-1) for im in levels]) if levels else np.zeros(1, np.uint8)
    return buf, p


def make_stereo_keys(k, keep):
    s = StereoKeys()
    s.n = int(len(k["x"]))
    s.x = keep.keep(f32(k["x"])).ctypes.data
    s.y = keep.keep(f32(k["y"])).ctypes.data
    s.octave = keep.keep(i32(k["octave"])).ctypes.data
    s.desc = keep.keep(u8(k["desc"])).ctypes.data
    return s


class MapPointsDev(C.Structure):
    _fields_ = [("n", C.c_int32), ("pos", C.c_void_p), ("normal", C.c_void_p), ("max_dist", C.c_void_p),
                ("min_dist", C.c_void_p), ("desc", C.c_void_p), ("locked", C.c_void_p), ("is_bad", C.c_void_p),
                ("in_frame", C.c_void_p)]


class KeypointsDev(C.Structure):  # lorb_keypoints with device pointers
    _fields_ = [("n", C.c_int32), ("x", C.c_void_p), ("y", C.c_void_p), ("octave", C.c_void_p),
                ("angle", C.c_void_p), ("u_right", C.c_void_p), ("desc", C.c_void_p)]


class LMOptions(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int32), ("function_tolerance", C.c_double),
                ("gradient_tolerance", C.c_double), ("parameter_tolerance", C.c_double),
                ("initial_trust_region_radius", C.c_double), ("max_trust_region_radius", C.c_double),
                ("min_trust_region_radius", C.c_double), ("min_relative_decrease", C.c_double),
                ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
                ("max_num_consecutive_invalid_steps", C.c_int32), ("jacobi_scaling", C.c_int32)]

    @classmethod
    def default(cls, **kw):
        o = cls(50, 1e-6, 1e-10, 1e-8, 1e4, 1e16, 1e-32, 1e-3, 1e-6, 1e32, 5, 1)
        for k, v in kw.items():
            setattr(o, k, v)
        return o


class BASummary(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("successful_steps", C.c_int32),
                ("termination", C.c_int32), ("pad_", C.c_int32),
                ("initial_cost", C.c_double), ("final_cost", C.c_double)]

    def as_dict(self):
        return {"iterations": self.iterations, "successful_steps": self.successful_steps,
                "termination": TERM_NAMES.get(self.termination, self.termination),
                "initial_cost": self.initial_cost, "final_cost": self.final_cost}


LM_STEP_NAMES = {0: "invalid", 1: "accepted", 2: "rejected", 3: "parameter_tol", 4: "function_tol"}
LM_TRACE_CAP = 64


class LMIteration(C.Structure):  # lorb_lm_iteration
    _fields_ = [("iteration", C.c_int32), ("outcome", C.c_int32), ("cost", C.c_double),
                ("model_cost_change", C.c_double), ("new_cost", C.c_double), ("radius", C.c_double),
                ("step_norm", C.c_double)]

    def as_dict(self):
        return {"iteration": self.iteration, "outcome": LM_STEP_NAMES.get(self.outcome, self.outcome),
                "cost": self.cost, "model_cost_change": self.model_cost_change, "new_cost": self.new_cost,
                "radius": self.radius, "step_norm": self.step_norm}


def trace_list(buf, n):
    return [buf[i].as_dict() for i in range(n)]


class PoseProblemBatch(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("res_off", i32p), ("intr", f32p), ("pose_init", f32p),
                ("pts3d", f32p), ("obs2d", f32p)]


class BAWindow(C.Structure):
    _fields_ = [("n_poses", C.c_int32), ("n_fixed", C.c_int32), ("n_points", C.c_int32),
                ("n_obs", C.c_int32), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("pose_init", f32p), ("fixed_pose", f32p), ("point_init", f32p),
                ("obs_point", i32p), ("obs_frame", i32p), ("obs_uv", f32p)]


# ------------------------------------------------------------------------------------------
def ptr(a, ctype):
    """Pointer to a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def make_frame_params(p):
    """dict (see synth.frame_params) -> FrameParams"""
    fp = FrameParams()
    for k in ("fx", "fy", "cx", "cy", "bf", "b", "min_x", "max_x", "min_y", "max_y",
              "grid_w_inv", "grid_h_inv", "log_scale_factor"):
        setattr(fp, k, float(p[k]))
    fp.n_levels = int(p["n_levels"])
    sf = np.zeros(LORB_MAX_LEVELS, np.float32)
    sf[: len(p["scale_factors"])] = p["scale_factors"]
    for i in range(LORB_MAX_LEVELS):
        fp.scale_factors[i] = float(sf[i])
    return fp


class KeepAlive(list):
    """Holds the numpy arrays a ctypes struct points into."""

    def keep(self, a):
        self.append(a)
        return a


def make_keypoints(kp, keep):
    k = Keypoints()
    k.n = int(len(kp["x"]))
    k.x = ptr(keep.keep(f32(kp["x"])), C.c_float)
    k.y = ptr(keep.keep(f32(kp["y"])), C.c_float)
    k.octave = ptr(keep.keep(i32(kp["octave"])), C.c_int32)
    k.angle = ptr(keep.keep(f32(kp["angle"])), C.c_float)
    k.u_right = ptr(keep.keep(f32(kp["u_right"])) if kp.get("u_right") is not None else None, C.c_float)
    k.desc = ptr(keep.keep(u8(kp["desc"])), C.c_uint8)
    return k


def make_last_frame(lf, keep):
    s = LastFrame()
    s.n = int(len(lf["has_mp"]))
    s.Tcw = ptr(keep.keep(f32(lf["Tcw"]).reshape(16)), C.c_float)
    s.has_mp = ptr(keep.keep(u8(lf["has_mp"])), C.c_uint8)
    s.outlier = ptr(keep.keep(u8(lf["outlier"])) if lf.get("outlier") is not None else None, C.c_uint8)
    s.mp_locked = ptr(keep.keep(u8(lf["mp_locked"])), C.c_uint8)
    s.mp_pos = ptr(keep.keep(f32(lf["mp_pos"])), C.c_float)
    s.mp_desc = ptr(keep.keep(u8(lf["mp_desc"])), C.c_uint8)
    s.octave = ptr(keep.keep(i32(lf["octave"])), C.c_int32)
    s.angle = ptr(keep.keep(f32(lf["angle"])), C.c_float)
    return s


def make_local_points(lp, keep):
    s = LocalPoints()
    s.n = int(len(lp["proj_x"]))
    s.track_in_view = ptr(keep.keep(u8(lp["track_in_view"])), C.c_uint8)
    s.is_bad = ptr(keep.keep(u8(lp["is_bad"])) if lp.get("is_bad") is not None else None, C.c_uint8)
    s.locked = ptr(keep.keep(u8(lp["locked"])), C.c_uint8)
    s.proj_x = ptr(keep.keep(f32(lp["proj_x"])), C.c_float)
    s.proj_y = ptr(keep.keep(f32(lp["proj_y"])), C.c_float)
    s.proj_xr = ptr(keep.keep(f32(lp["proj_xr"])), C.c_float)
    s.pred_level = ptr(keep.keep(i32(lp["pred_level"])), C.c_int32)
    s.view_cos = ptr(keep.keep(f32(lp["view_cos"])), C.c_float)
    s.desc = ptr(keep.keep(u8(lp["desc"])), C.c_uint8)
    return s


def make_frustum_points(fpts, keep):
    s = FrustumPoints()
    s.n = int(len(fpts["max_dist"]))
    s.pos = ptr(keep.keep(f32(fpts["pos"])), C.c_float)
    s.normal = ptr(keep.keep(f32(fpts["normal"])), C.c_float)
    s.max_dist = ptr(keep.keep(f32(fpts["max_dist"])), C.c_float)
    s.min_dist = ptr(keep.keep(f32(fpts["min_dist"])), C.c_float)
    return s


def make_pose_batch(pb, keep):
    s = PoseProblemBatch()
    s.n_frames = int(len(pb["res_off"]) - 1)
    s.res_off = ptr(keep.keep(i32(pb["res_off"])), C.c_int32)
    s.intr = ptr(keep.keep(f32(pb["intr"])), C.c_float)
    s.pose_init = ptr(keep.keep(f32(pb["pose_init"])), C.c_float)
    s.pts3d = ptr(keep.keep(f32(pb["pts3d"])), C.c_float)
    s.obs2d = ptr(keep.keep(f32(pb["obs2d"])), C.c_float)
    return s


class BAWindowDev(C.Structure):
    """lorb_ba_window_dev: one window whose arrays live in device memory (device pointers)."""
    _fields_ = [("n_poses", C.c_int32), ("n_fixed", C.c_int32), ("max_points", C.c_int32), ("max_obs", C.c_int32),
                ("d_n_points", C.c_void_p), ("d_n_obs", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("d_pose_init", C.c_void_p), ("d_fixed_pose", C.c_void_p), ("d_point_init", C.c_void_p),
                ("d_obs_point", C.c_void_p), ("d_obs_frame", C.c_void_p), ("d_obs_uv", C.c_void_p)]


class MapInit(C.Structure):
    """lorb_map_init: the local map's initial window (host arrays)."""
    _fields_ = [("n_window", C.c_int32), ("n_fixed", C.c_int32), ("max_points", C.c_int32), ("max_obs", C.c_int32),
                ("max_keypoints", C.c_int32), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("pose", f32p), ("fixed_pose", f32p), ("n_points", C.c_int32), ("n_obs", C.c_int32),
                ("point", f32p), ("point_desc", C.POINTER(C.c_uint8)), ("obs_point", i32p), ("obs_kf", i32p),
                ("obs_uv", f32p)]


class MapKeyframe(C.Structure):
    """lorb_map_keyframe: one map's keyframe of a lorb_map_group step (host pose / Tcw, device keypoints)."""
    _fields_ = [("frame", C.POINTER(FrameParams)), ("pose", f32p), ("Tcw", f32p), ("n", C.c_int32),
                ("d_desc", C.c_void_p), ("d_x", C.c_void_p), ("d_y", C.c_void_p), ("d_depth", C.c_void_p)]


class MapState(C.Structure):
    """lorb_map_state: host buffers lorb_map_read fills (NULL = skip)."""
    _fields_ = [("point", f32p), ("point_desc", C.POINTER(C.c_uint8)), ("obs_point", i32p), ("obs_kf", i32p),
                ("obs_uv", f32p), ("obs_frame", i32p), ("pose", f32p), ("fixed_pose", f32p), ("match_train", i32p),
                ("summary", C.POINTER(BASummary))]


def make_windows(wins, keep):
    arr = (BAWindow * max(1, len(wins)))()
    for i, w in enumerate(wins):
        s = arr[i]
        s.n_poses = int(len(w["pose_init"]))
        s.n_fixed = int(len(w["fixed_pose"]))
        s.n_points = int(len(w["point_init"]))
        s.n_obs = int(len(w["obs_point"]))
        s.fx, s.fy, s.cx, s.cy = (float(v) for v in w["intr"])
        s.pose_init = ptr(keep.keep(f32(w["pose_init"])), C.c_float)
        s.fixed_pose = ptr(keep.keep(f32(w["fixed_pose"]).reshape(-1, 6)), C.c_float)
        s.point_init = ptr(keep.keep(f32(w["point_init"])), C.c_float)
        s.obs_point = ptr(keep.keep(i32(w["obs_point"])), C.c_int32)
        s.obs_frame = ptr(keep.keep(i32(w["obs_frame"])), C.c_int32)
        s.obs_uv = ptr(keep.keep(f32(w["obs_uv"])), C.c_float)
    return arr
