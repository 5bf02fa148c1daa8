"""Loader + thin ctypes bindings of liblorb.so (include/lorb_c.h).

The product path is the HIP library.  There is no CPU fallback: if liblorb.so is missing
or no MI355X is visible, every call raises.
"""
import ctypes as C
import os

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LORB_LIB_PATH") or os.path.join(_HERE, "liblorb.so")  # override: diagnostics only
_lib = None


class LorbError(RuntimeError):
    pass


def lib():
    """Load the in-tree liblorb.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LorbError(f"{LIB_PATH} not built: run `make -C lorb_slam_amd/csrc` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        L.lorb_last_error.restype = C.c_char_p
        L.lorb_last_error.argtypes = [C.c_void_p]
        for name in ("lorb_create", "lorb_destroy", "lorb_sync", "lorb_malloc", "lorb_free",
                     "lorb_memcpy_h2d", "lorb_memcpy_d2h", "lorb_memset_dev", "lorb_timer_mark",
                     "lorb_timer_elapsed_ms", "lorb_device_count", "lorb_abi_version"):
            getattr(L, name).restype = C.c_int
        _lib = L
    return _lib


def device_count():
    n = C.c_int(0)
    rc = lib().lorb_device_count(C.byref(n))
    return n.value if rc == 0 else 0


class Context:
    """One lorb_ctx (one HIP stream) on one device.  Not thread-safe (one per thread)."""

    def __init__(self, device=0):
        self._p = C.c_void_p()
        rc = lib().lorb_create(C.c_int(device), C.byref(self._p))
        if rc != 0:
            raise LorbError(f"lorb_create(device={device}) failed rc={rc}: no usable HIP device")
        self.device = device

    @property
    def handle(self):
        return self._p

    def check(self, rc, what):
        if rc != 0:
            msg = lib().lorb_last_error(self._p)
            raise LorbError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")

    def close(self):
        if self._p:
            lib().lorb_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self.check(lib().lorb_sync(self._p), "lorb_sync")

    # device memory -----------------------------------------------------------------------
    def malloc(self, nbytes):
        p = C.c_void_p()
        self.check(lib().lorb_malloc(self._p, C.byref(p), C.c_size_t(nbytes)), "lorb_malloc")
        return p

    def free(self, p):
        self.check(lib().lorb_free(self._p, p), "lorb_free")

    def to_device(self, arr):
        arr = np.ascontiguousarray(arr)
        p = self.malloc(max(arr.nbytes, 16))
        self.check(lib().lorb_memcpy_h2d(self._p, p, arr.ctypes.data_as(C.c_void_p), C.c_size_t(arr.nbytes)), "h2d")
        return DeviceArray(self, p, arr.shape, arr.dtype)

    def empty(self, shape, dtype):
        dt = np.dtype(dtype)
        n = int(np.prod(shape)) * dt.itemsize
        return DeviceArray(self, self.malloc(max(n, 16)), tuple(np.atleast_1d(shape)) if np.ndim(shape) else (int(shape),), dt)

    def timer_mark(self, slot):
        self.check(lib().lorb_timer_mark(self._p, C.c_int(slot)), "timer_mark")

    def timer_ms(self, a, b):
        ms = C.c_float(0)
        self.check(lib().lorb_timer_elapsed_ms(self._p, C.c_int(a), C.c_int(b), C.byref(ms)), "timer")
        return ms.value

    # matcher -------------------------------------------------------------------------------
    def bf_top2(self, q_list, t_list, t_level_list=None):
        """Batched a5-with-unbounded-window: lists of (Nq_i x 32) / (Nt_i x 32) uint8 arrays."""
        q = np.ascontiguousarray(np.concatenate(q_list) if len(q_list) else np.zeros((0, 32), np.uint8), np.uint8)
        t = np.ascontiguousarray(np.concatenate(t_list) if len(t_list) else np.zeros((0, 32), np.uint8), np.uint8)
        q_off = np.concatenate([[0], np.cumsum([len(a) for a in q_list])]).astype(np.int32)
        t_off = np.concatenate([[0], np.cumsum([len(a) for a in t_list])]).astype(np.int32)
        tl = None
        if t_level_list is not None:
            tl = np.ascontiguousarray(np.concatenate(t_level_list), np.int32)
        nq = len(q)
        out = {k: np.zeros(max(nq, 1), np.int32) for k in ("best_idx", "best_dist", "best_level", "second_dist", "second_level")}
        acc = np.zeros(max(nq, 1), np.uint8)
        self.check(lib().lorb_bf_top2(
            self._p, C.c_int32(len(q_list)), A.ptr(q, C.c_uint8), A.ptr(q_off, C.c_int32), A.ptr(t, C.c_uint8),
            A.ptr(t_off, C.c_int32), A.ptr(tl, C.c_int32), A.ptr(out["best_idx"], C.c_int32),
            A.ptr(out["best_dist"], C.c_int32), A.ptr(out["best_level"], C.c_int32),
            A.ptr(out["second_dist"], C.c_int32), A.ptr(out["second_level"], C.c_int32),
            A.ptr(acc, C.c_uint8)), "lorb_bf_top2")
        out["accepted"] = acc
        return {k: v[:nq] for k, v in out.items()}, q_off

    def bf_match(self, q_list, t_list):
        q = np.ascontiguousarray(np.concatenate(q_list) if len(q_list) else np.zeros((0, 32), np.uint8), np.uint8)
        t = np.ascontiguousarray(np.concatenate(t_list) if len(t_list) else np.zeros((0, 32), np.uint8), np.uint8)
        q_off = np.concatenate([[0], np.cumsum([len(a) for a in q_list])]).astype(np.int32)
        t_off = np.concatenate([[0], np.cumsum([len(a) for a in t_list])]).astype(np.int32)
        nq = len(q)
        cc_t = np.zeros(max(nq, 1), np.int32); cc_d = np.zeros(max(nq, 1), np.int32); mt = np.zeros(max(nq, 1), np.int32)
        nm = np.zeros(max(len(q_list), 1), np.int32)
        self.check(lib().lorb_bf_match(
            self._p, C.c_int32(len(q_list)), A.ptr(q, C.c_uint8), A.ptr(q_off, C.c_int32), A.ptr(t, C.c_uint8),
            A.ptr(t_off, C.c_int32), A.ptr(cc_t, C.c_int32), A.ptr(cc_d, C.c_int32), A.ptr(mt, C.c_int32),
            A.ptr(nm, C.c_int32)), "lorb_bf_match")
        return dict(cc_train=cc_t[:nq], cc_dist=cc_d[:nq], match_train=mt[:nq], n_matches=nm[: len(q_list)]), q_off


def _bf_match_sharded(self, comm, q_list, q_base, t_list):
    """lorb_bf_match_sharded_dev: this rank's query rows of every problem (q_list[p] starts at
    global query q_base[p]) against all trains; returns local outputs + global match counts."""
    q = np.ascontiguousarray(np.concatenate(q_list) if len(q_list) else np.zeros((0, 32), np.uint8), np.uint8)
    t = np.ascontiguousarray(np.concatenate(t_list) if len(t_list) else np.zeros((0, 32), np.uint8), np.uint8)
    q_off = np.concatenate([[0], np.cumsum([len(a) for a in q_list])]).astype(np.int32)
    t_off = np.concatenate([[0], np.cumsum([len(a) for a in t_list])]).astype(np.int32)
    qb = np.ascontiguousarray(q_base, np.int32)
    nq, npb = len(q), len(q_list)
    dq, dt = self.to_device(q if nq else np.zeros((1, 32), np.uint8)), self.to_device(t if len(t) else np.zeros((1, 32), np.uint8))
    outs = [self.empty(max(nq, 1), np.int32) for _ in range(3)]
    nm = self.empty(max(npb, 1), np.int32)
    self.check(lib().lorb_bf_match_sharded_dev(
        self._p, comm.handle, C.c_int32(npb), dq.as_ptr(C.c_uint8), A.ptr(q_off, C.c_int32), A.ptr(qb, C.c_int32),
        dt.as_ptr(C.c_uint8), A.ptr(t_off, C.c_int32), *[o.as_ptr(C.c_int32) for o in outs], nm.as_ptr(C.c_int32)),
        "lorb_bf_match_sharded_dev")
    res = dict(cc_train=outs[0].numpy()[:nq], cc_dist=outs[1].numpy()[:nq], match_train=outs[2].numpy()[:nq],
               n_matches=nm.numpy()[:npb])
    for a in (dq, dt, nm, *outs):
        a.free()
    return res


Context.bf_match_sharded = _bf_match_sharded


def _compute_descriptor(self, d_off, desc):
    """lorb_compute_descriptor: best candidate index per map point (-1: empty) + its descriptor."""
    d_off = np.ascontiguousarray(d_off, np.int32)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(d_off) - 1
    best = np.zeros(max(n, 1), np.int32)
    out = np.zeros((max(n, 1), 32), np.uint8)
    self.check(lib().lorb_compute_descriptor(self._p, C.c_int32(n), A.ptr(d_off, C.c_int32),
                                             A.ptr(desc if len(desc) else np.zeros((1, 32), np.uint8), C.c_uint8),
                                             A.ptr(best, C.c_int32), A.ptr(out, C.c_uint8)), "lorb_compute_descriptor")
    return best[:n], out[:n]


Context.compute_descriptor = _compute_descriptor


class DeviceArray:
    def __init__(self, ctx, ptr_, shape, dtype):
        self.ctx, self.ptr, self.shape, self.dtype = ctx, ptr_, tuple(shape), np.dtype(dtype)

    @property
    def nbytes(self):
        return int(np.prod(self.shape)) * self.dtype.itemsize

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        if self.nbytes:
            self.ctx.check(lib().lorb_memcpy_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p), self.ptr,
                                                 C.c_size_t(self.nbytes)), "d2h")
        return out

    def free(self):
        if self.ptr:
            self.ctx.free(self.ptr)
            self.ptr = None

    def as_ptr(self, ctype):
        return C.cast(self.ptr, C.POINTER(ctype))


# ---- bundle adjustment ---------------------------------------------------------------------
def _ba_pose_only(self, pb, opt=None):
    keep = A.KeepAlive()
    s = A.make_pose_batch(pb, keep)
    opt = opt or A.LMOptions.default()
    nf = s.n_frames
    pose = np.zeros((max(nf, 1), 6)); T = np.zeros((max(nf, 1), 4, 4), np.float32)
    summ = (A.BASummary * max(1, nf))()
    self.check(lib().lorb_ba_pose_only(self._p, C.byref(s), C.byref(opt), A.ptr(pose, C.c_double),
                                       A.ptr(T, C.c_float), summ), "lorb_ba_pose_only")
    return pose[:nf], T[:nf], [summ[i].as_dict() for i in range(nf)]


def _ba_local(self, wins, opt=None):
    keep = A.KeepAlive()
    arr = A.make_windows(wins, keep)
    opt = opt or A.LMOptions.default()
    poses = [np.zeros((len(w["pose_init"]), 6)) for w in wins]
    pts = [np.zeros((len(w["point_init"]), 3)) for w in wins]
    pp = (A.f64p * max(1, len(wins)))(*[A.ptr(p, C.c_double) for p in poses])
    qp = (A.f64p * max(1, len(wins)))(*[A.ptr(p, C.c_double) for p in pts])
    summ = (A.BASummary * max(1, len(wins)))()
    self.check(lib().lorb_ba_local(self._p, C.c_int32(len(wins)), arr, C.byref(opt), pp, qp, summ), "lorb_ba_local")
    return poses, pts, [summ[i].as_dict() for i in range(len(wins))]


HOST_ALLREDUCE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64, C.c_int32)
OP_SUM, OP_MAX, OP_MIN = 0, 1, 2


def unique_id():
    """RCCL unique id (bytes) -- create on rank 0, distribute out of band."""
    buf = (C.c_uint8 * 128)()
    rc = lib().lorb_comm_unique_id(buf)
    if rc != 0:
        raise LorbError(f"lorb_comm_unique_id failed rc={rc}")
    return bytes(buf)


class Comm:
    """lorb_comm: the multi-GPU exchange of the sharded local BA (include/lorb_c.h).

    Comm.rccl(ctx, world, rank, uid): ncclAllReduce on the context stream (one process per GPU).
    Comm.host(ctx, world, rank, fn):  fn(np.ndarray float64 view, op) all-reduces in place over
    the ranks by any host transport (tests: torch.distributed gloo)."""

    def __init__(self, ctx, handle, keep=None):
        self.ctx, self._p, self._keep = ctx, handle, keep

    @classmethod
    def rccl(cls, ctx, world, rank, uid):
        h = C.c_void_p()
        idb = (C.c_uint8 * 128).from_buffer_copy(uid)
        ctx.check(lib().lorb_comm_init_rccl(ctx.handle, C.c_int32(world), C.c_int32(rank), idb, C.byref(h)),
                  "lorb_comm_init_rccl")
        return cls(ctx, h)

    @classmethod
    def host(cls, ctx, world, rank, fn):
        def cb(_user, buf, n, op):
            try:
                fn(np.ctypeslib.as_array(buf, shape=(int(n),)), int(op))
                return 0
            except Exception:  # noqa: BLE001 -- reported to the library as a transport failure
                import traceback
                traceback.print_exc()
                return 1
        cfn = HOST_ALLREDUCE(cb)
        h = C.c_void_p()
        ctx.check(lib().lorb_comm_init_host(ctx.handle, C.c_int32(world), C.c_int32(rank), cfn, None, C.byref(h)),
                  "lorb_comm_init_host")
        return cls(ctx, h, keep=cfn)

    @property
    def handle(self):
        return self._p

    def size(self):
        """(nranks, rank) as the communicator itself reports them (ncclCommCount for RCCL)."""
        n, r = C.c_int32(0), C.c_int32(0)
        self.ctx.check(lib().lorb_comm_size(self._p, C.byref(n), C.byref(r)), "lorb_comm_size")
        return n.value, r.value

    def close(self):
        if self._p:
            lib().lorb_comm_destroy(self._p)
            self._p = C.c_void_p()


class BAPlan:
    """Device-resident plan (lorb_ba_plan_*): upload + Schur structure once, solve many times.
    With `comm`, `wins` are this rank's shards (lorb_ba_plan_create_sharded)."""

    def __init__(self, ctx, wins, comm=None):
        self.ctx = ctx
        self.wins = wins
        self.comm = comm
        self._keep = A.KeepAlive()
        arr = A.make_windows(wins, self._keep)
        self._p = C.c_void_p()
        if comm is None:
            ctx.check(lib().lorb_ba_plan_create(ctx.handle, C.c_int32(len(wins)), arr, C.byref(self._p)),
                      "lorb_ba_plan_create")
        else:
            ctx.check(lib().lorb_ba_plan_create_sharded(ctx.handle, comm.handle, C.c_int32(len(wins)), arr,
                                                        C.byref(self._p)), "lorb_ba_plan_create_sharded")

    def solve(self, opt=None):
        opt = opt or A.LMOptions.default()
        self.ctx.check(lib().lorb_ba_plan_solve(self._p, C.byref(opt)), "lorb_ba_plan_solve")

    def read(self):
        wins = self.wins
        poses = [np.zeros((len(w["pose_init"]), 6)) for w in wins]
        pts = [np.zeros((len(w["point_init"]), 3)) for w in wins]
        pp = (A.f64p * max(1, len(wins)))(*[A.ptr(p, C.c_double) for p in poses])
        qp = (A.f64p * max(1, len(wins)))(*[A.ptr(p, C.c_double) for p in pts])
        summ = (A.BASummary * max(1, len(wins)))()
        self.ctx.check(lib().lorb_ba_plan_read(self._p, pp, qp, summ), "lorb_ba_plan_read")
        return poses, pts, [summ[i].as_dict() for i in range(len(wins))]

    def trace(self, w=0):
        """lorb_ba_plan_trace: the last solve's per-iteration records of window w"""
        buf, n = (A.LMIteration * A.LM_TRACE_CAP)(), C.c_int32()
        self.ctx.check(lib().lorb_ba_plan_trace(self._p, C.c_int32(w), buf, C.c_int32(A.LM_TRACE_CAP), C.byref(n)),
                       "lorb_ba_plan_trace")
        return A.trace_list(buf, n.value)

    def info(self):
        """lorb_ba_plan_info: structure of the plan and the Cholesky kernel of the last solve."""
        v = (C.c_int32 * 11)()
        self.ctx.check(lib().lorb_ba_plan_info(self._p, v, C.c_int32(11)), "lorb_ba_plan_info")
        keys = ("band", "cholesky", "blocks", "point_groups", "observations", "points", "cameras", "reordered",
                "point_major", "red_threads", "partial_runs")
        return dict(zip(keys, [int(x) for x in v]))

    def close(self):
        if self._p:
            lib().lorb_ba_plan_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BASolver:
    """lorb_ba_solver: BA::LocalPoseOptimization for a caller that gathers a new window every call
    (the drop-in's path, include/lorb/adapters.hpp); device-built plans stay resident across calls."""

    INFO_KEYS = ("resident_plans", "plan_creations", "host_plan_fallback", "band", "cholesky", "reordered")

    def __init__(self, ctx):
        self.ctx = ctx
        self._p = C.c_void_p()
        ctx.check(lib().lorb_ba_solver_create(ctx.handle, C.byref(self._p)), "lorb_ba_solver_create")

    def prepare(self, w):
        """ctypes window of one dict window (kept alive by the returned tuple) and its output arrays"""
        keep = A.KeepAlive()
        arr = A.make_windows([w], keep)
        pose = np.zeros((len(w["pose_init"]), 6))
        pts = np.zeros((len(w["point_init"]), 3))
        return (arr, keep, pose, pts, A.BASummary())

    def solve_prepared(self, prep, opt):
        arr, _, pose, pts, summ = prep
        self.ctx.check(lib().lorb_ba_solver_solve(self._p, arr, C.byref(opt), A.ptr(pose, C.c_double),
                                                  A.ptr(pts, C.c_double), C.byref(summ)), "lorb_ba_solver_solve")
        return pose, pts, summ.as_dict()

    def solve(self, w, opt=None):
        """(poses n_poses x 6, points n_points x 3, summary) of one window dict"""
        return self.solve_prepared(self.prepare(w), opt or A.LMOptions.default())

    def trace(self):
        """lorb_ba_solver_trace: the last call's per-iteration records"""
        buf, n = (A.LMIteration * A.LM_TRACE_CAP)(), C.c_int32()
        self.ctx.check(lib().lorb_ba_solver_trace(self._p, buf, C.c_int32(A.LM_TRACE_CAP), C.byref(n)),
                       "lorb_ba_solver_trace")
        return A.trace_list(buf, n.value)

    def info(self):
        v = (C.c_int32 * 6)()
        self.ctx.check(lib().lorb_ba_solver_info(self._p, v, C.c_int32(6)), "lorb_ba_solver_info")
        return dict(zip(self.INFO_KEYS, [int(x) for x in v]))

    def close(self):
        if self._p:
            lib().lorb_ba_solver_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BAPlanDev(BAPlan):
    """Device-built plan (lorb_ba_plan_create_dev / _update_dev) of one window held in device
    memory: `arrays` is a dict of DeviceArrays (n_points, n_obs: 1 int each; pose_init, fixed_pose,
    point_init, obs_point, obs_frame, obs_uv), `intr` = (fx, fy, cx, cy)."""

    def __init__(self, ctx, arrays, n_poses, n_fixed, intr, comm=None):  # noqa: D107 -- BAPlan's fields
        self.ctx, self.comm, self._keep = ctx, comm, A.KeepAlive()
        self._p = C.c_void_p()
        self.n_poses, self.n_fixed = n_poses, n_fixed
        self.win = self._window(arrays, intr)
        if comm is None:
            ctx.check(lib().lorb_ba_plan_create_dev(ctx.handle, C.byref(self.win), C.byref(self._p)),
                      "lorb_ba_plan_create_dev")
        else:  # this rank's shard; every build is collective (lorb_ba_plan_create_sharded_dev)
            ctx.check(lib().lorb_ba_plan_create_sharded_dev(ctx.handle, comm.handle, C.byref(self.win), C.byref(self._p)),
                      "lorb_ba_plan_create_sharded_dev")

    @staticmethod
    def upload(ctx, w, extra_points=0, extra_obs=0):
        """device arrays of a window dict (synth.ba_window / shard.shard_window) with spare capacity"""
        P, K = len(w["point_init"]), len(w["obs_point"])

        def pad(a, n):
            a = np.asarray(a)
            return np.concatenate([a, np.zeros((n - len(a),) + a.shape[1:], a.dtype)])
        return dict(n_points=ctx.to_device(np.array([P], np.int32)), n_obs=ctx.to_device(np.array([K], np.int32)),
                    pose_init=ctx.to_device(A.f32(w["pose_init"]).reshape(-1, 6)),
                    fixed_pose=ctx.to_device(A.f32(w["fixed_pose"]).reshape(-1, 6)),
                    point_init=ctx.to_device(pad(A.f32(w["point_init"]).reshape(-1, 3), max(P + extra_points, 1))),
                    obs_point=ctx.to_device(pad(A.i32(w["obs_point"]), max(K + extra_obs, 1))),
                    obs_frame=ctx.to_device(pad(A.i32(w["obs_frame"]), max(K + extra_obs, 1))),
                    obs_uv=ctx.to_device(pad(A.f32(w["obs_uv"]).reshape(-1, 2), max(K + extra_obs, 1))))

    def _window(self, a, intr):
        self.arrays = a
        w = A.BAWindowDev()
        w.n_poses, w.n_fixed = self.n_poses, self.n_fixed
        w.max_points, w.max_obs = a["point_init"].shape[0], a["obs_point"].shape[0]
        w.d_n_points, w.d_n_obs = a["n_points"].ptr, a["n_obs"].ptr
        w.fx, w.fy, w.cx, w.cy = (float(v) for v in intr)
        for k in ("pose_init", "fixed_pose", "point_init", "obs_point", "obs_frame", "obs_uv"):
            setattr(w, "d_" + k, a[k].ptr)
        return w

    def update(self, arrays=None, intr=None):
        if arrays is not None:
            self.win = self._window(arrays, intr if intr is not None else (self.win.fx, self.win.fy, self.win.cx, self.win.cy))
        self.ctx.check(lib().lorb_ba_plan_update_dev(self._p, C.byref(self.win)), "lorb_ba_plan_update_dev")

    def read(self):
        info = self.info()
        poses = np.zeros((self.n_poses, 6)); pts = np.zeros((max(info["points"], 1), 3))
        pp = (A.f64p * 1)(A.ptr(poses, C.c_double))
        qp = (A.f64p * 1)(A.ptr(pts, C.c_double))
        summ = (A.BASummary * 1)()
        self.ctx.check(lib().lorb_ba_plan_read(self._p, pp, qp, summ), "lorb_ba_plan_read")
        return [poses], [pts[:info["points"]]], [summ[0].as_dict()]

    def result_dev(self, d_pose, d_points):
        self.ctx.check(lib().lorb_ba_plan_result_dev(self._p, d_pose.ptr if d_pose is not None else None,
                                                     d_points.ptr if d_points is not None else None),
                       "lorb_ba_plan_result_dev")


class LocalMap:
    """lorb_map: the HBM-resident local map and its chained LocalMapping step (include/lorb_c.h;
    SURVEY §8 a17 full step).  `init`: dict(pose_init W x 6, fixed_pose F x 6, point_init, point_desc,
    obs_point, obs_kf (keyframe ids in [-F, W)), obs_uv, intr) -- synth.mapping_sequence()["init"]."""

    COUNT_KEYS = ("points", "observations", "t0", "keypoints", "new_points", "new_observations", "matches", "window",
                  "overlapped_steps")

    def __init__(self, ctx, init, max_points=None, max_obs=None, max_keypoints=4096):
        self.ctx, self._keep = ctx, A.KeepAlive()
        k = self._keep.keep
        s = A.MapInit()
        s.n_window, s.n_fixed = len(init["pose_init"]), len(init["fixed_pose"])
        s.n_points, s.n_obs = len(init["point_init"]), len(init["obs_point"])
        s.max_points = int(max_points or 2 * s.n_points + 8 * max_keypoints)
        s.max_obs = int(max_obs or 2 * s.n_obs + 8 * max_keypoints)
        s.max_keypoints = int(max_keypoints)
        s.fx, s.fy, s.cx, s.cy = (float(v) for v in init["intr"])
        s.pose = A.ptr(k(A.f32(init["pose_init"])), C.c_float)
        s.fixed_pose = A.ptr(k(A.f32(init["fixed_pose"]).reshape(-1, 6)), C.c_float)
        s.point = A.ptr(k(A.f32(init["point_init"])), C.c_float)
        s.point_desc = A.ptr(k(A.u8(init["point_desc"])), C.c_uint8)
        s.obs_point = A.ptr(k(A.i32(init["obs_point"])), C.c_int32)
        s.obs_kf = A.ptr(k(A.i32(init["obs_kf"])), C.c_int32)
        s.obs_uv = A.ptr(k(A.f32(init["obs_uv"])), C.c_float)
        self.W, self.F, self.max_keypoints = s.n_window, s.n_fixed, s.max_keypoints
        self._p = C.c_void_p()
        ctx.check(lib().lorb_map_create(ctx.handle, C.byref(s), C.byref(self._p)), "lorb_map_create")
        self._keep.clear()

    def set_overlap(self, enable=True):
        """lorb_map_set_overlap: step t+1's match + append on the map's own stream under step t's
        solve.  The keyframe arrays of step_dev must then be complete when it is called."""
        self.ctx.check(lib().lorb_map_set_overlap(self._p, C.c_int32(1 if enable else 0)), "lorb_map_set_overlap")

    def step_dev(self, fp, pose, Tcw, n, d_desc, d_x, d_y, d_depth, opt=None):
        """one step on device-resident keypoints (DeviceArrays); fp: FrameParams"""
        opt = opt or A.LMOptions.default()
        pose = A.f32(pose).reshape(6); T = A.f32(Tcw).reshape(16)
        self.ctx.check(lib().lorb_map_step_dev(self._p, C.byref(fp), A.ptr(pose, C.c_float), A.ptr(T, C.c_float),
                                               C.c_int32(n), d_desc.ptr, d_x.ptr, d_y.ptr, d_depth.ptr, C.byref(opt)),
                       "lorb_map_step_dev")

    def step(self, fp, kf, opt=None):
        """upload one keyframe (synth.mapping_sequence()["steps"][i]) and step"""
        fps = A.make_frame_params(fp) if isinstance(fp, dict) else fp
        arrs = [self.ctx.to_device(A.u8(kf["desc"])), self.ctx.to_device(A.f32(kf["x"])),
                self.ctx.to_device(A.f32(kf["y"])), self.ctx.to_device(A.f32(kf["depth"]))]
        try:
            self.step_dev(fps, kf["pose"], kf["Tcw"], len(kf["x"]), *arrs, opt=opt)
            self.ctx.sync()
        finally:
            for a in arrs:
                a.free()

    def counts(self):
        v = (C.c_int32 * 9)()
        self.ctx.check(lib().lorb_map_counts(self._p, v, C.c_int32(9)), "lorb_map_counts")
        return dict(zip(self.COUNT_KEYS, [int(x) for x in v]))

    def read(self):
        c = self.counts()
        P, K = c["points"], c["observations"]
        out = dict(point=np.zeros((max(P, 1), 3), np.float32), point_desc=np.zeros((max(P, 1), 32), np.uint8),
                   obs_point=np.zeros(max(K, 1), np.int32), obs_kf=np.zeros(max(K, 1), np.int32),
                   obs_uv=np.zeros((max(K, 1), 2), np.float32), obs_frame=np.zeros(max(K, 1), np.int32),
                   pose=np.zeros((self.W, 6), np.float32), fixed_pose=np.zeros((max(self.F, 1), 6), np.float32),
                   match_train=np.zeros(max(c["keypoints"], 1), np.int32))
        summ = A.BASummary()
        st = A.MapState()
        st.point = A.ptr(out["point"], C.c_float); st.point_desc = A.ptr(out["point_desc"], C.c_uint8)
        st.obs_point = A.ptr(out["obs_point"], C.c_int32); st.obs_kf = A.ptr(out["obs_kf"], C.c_int32)
        st.obs_uv = A.ptr(out["obs_uv"], C.c_float); st.obs_frame = A.ptr(out["obs_frame"], C.c_int32)
        st.pose = A.ptr(out["pose"], C.c_float); st.fixed_pose = A.ptr(out["fixed_pose"], C.c_float)
        st.match_train = A.ptr(out["match_train"], C.c_int32); st.summary = C.pointer(summ)
        self.ctx.check(lib().lorb_map_read(self._p, C.byref(st)), "lorb_map_read")
        for key, n in (("point", P), ("point_desc", P), ("obs_point", K), ("obs_kf", K), ("obs_uv", K),
                       ("obs_frame", K), ("fixed_pose", self.F), ("match_train", c["keypoints"])):
            out[key] = out[key][:n]
        out["summary"] = summ.as_dict()
        out.update(c)
        return out

    def trace(self):
        """the last step's LM records (lorb_ba_plan_trace of the map's plan)"""
        p = C.c_void_p()
        self.ctx.check(lib().lorb_map_plan(self._p, C.byref(p)), "lorb_map_plan")
        buf, n = (A.LMIteration * A.LM_TRACE_CAP)(), C.c_int32()
        self.ctx.check(lib().lorb_ba_plan_trace(p, C.c_int32(0), buf, C.c_int32(A.LM_TRACE_CAP), C.byref(n)),
                       "lorb_ba_plan_trace")
        return A.trace_list(buf, n.value)

    def plan_info(self):
        p = C.c_void_p()
        self.ctx.check(lib().lorb_map_plan(self._p, C.byref(p)), "lorb_map_plan")
        v = (C.c_int32 * 8)()
        self.ctx.check(lib().lorb_ba_plan_info(p, v, C.c_int32(8)), "lorb_ba_plan_info")
        keys = ("band", "cholesky", "blocks", "point_groups", "observations", "points", "cameras", "reordered")
        return dict(zip(keys, [int(x) for x in v]))

    def close(self):
        if self._p:
            lib().lorb_map_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BAGroup:
    """lorb_ba_group: the LM solves of several plans on one context as one set of launches (each
    plan's results bit-identical to its own solve).  The plans are not owned and must outlive it."""

    def __init__(self, ctx, plans):
        self.ctx, self.plans = ctx, list(plans)
        arr = (C.c_void_p * len(self.plans))(*[p._p for p in self.plans])
        self._p = C.c_void_p()
        ctx.check(lib().lorb_ba_group_create(ctx.handle, C.c_int32(len(self.plans)), arr, C.byref(self._p)),
                  "lorb_ba_group_create")

    def solve(self, opt=None):
        opt = opt or A.LMOptions.default()
        self.ctx.check(lib().lorb_ba_group_solve(self._p, C.byref(opt)), "lorb_ba_group_solve")

    def info(self):
        v = (C.c_int32 * 3)()
        self.ctx.check(lib().lorb_ba_group_info(self._p, v, C.c_int32(3)), "lorb_ba_group_info")
        return dict(zip(("plans", "fused_solves", "captures"), [int(x) for x in v]))

    def close(self):
        if self._p:
            lib().lorb_ba_group_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MapGroup:
    """lorb_map_group: several LocalMaps on one context stepped together -- per map steps 1-3 and
    the plan build, then one BA solve over all of their plans (lorb_ba_group), then the write-backs.
    Each map's state is bit-identical to stepping it alone."""

    def __init__(self, maps):
        self.maps = list(maps)
        self.ctx = self.maps[0].ctx
        arr = (C.c_void_p * len(self.maps))(*[m._p for m in self.maps])
        self._p = C.c_void_p()
        self.ctx.check(lib().lorb_map_group_create(C.c_int32(len(self.maps)), arr, C.byref(self._p)),
                       "lorb_map_group_create")

    def step_dev(self, fp, kfs, opt=None):
        """kfs: per map (pose, Tcw, n, d_desc, d_x, d_y, d_depth) with DeviceArrays; fp: FrameParams"""
        opt = opt or A.LMOptions.default()
        arr = (A.MapKeyframe * len(self.maps))()
        keep = []
        for k, (pose, Tcw, n, dd, dx, dy, dz) in zip(arr, kfs):
            pose = A.f32(pose).reshape(6); T = A.f32(Tcw).reshape(16)
            keep += [pose, T]
            k.frame = C.pointer(fp); k.pose = A.ptr(pose, C.c_float); k.Tcw = A.ptr(T, C.c_float); k.n = int(n)
            k.d_desc, k.d_x, k.d_y, k.d_depth = dd.ptr, dx.ptr, dy.ptr, dz.ptr
        self.ctx.check(lib().lorb_map_group_step_dev(self._p, arr, C.byref(opt)), "lorb_map_group_step_dev")

    def info(self):
        v = (C.c_int32 * 4)()
        self.ctx.check(lib().lorb_map_group_info(self._p, v, C.c_int32(4)), "lorb_map_group_info")
        return dict(zip(("maps", "plan_groups", "fused_steps", "captures"), [int(x) for x in v]))

    def close(self):
        if self._p:
            lib().lorb_map_group_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


Context.ba_pose_only = _ba_pose_only
Context.ba_local = _ba_local

from . import window as _window  # noqa: E402,F401  (binds the windowed-matcher methods onto Context)
