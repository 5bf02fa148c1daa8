"""GPU parity: lorb_ba_solver (the drop-in BA::LocalPoseOptimization path, src/bundle_adjust.cpp:207-330,
with device-built plans resident across calls) vs the oracle's or_ba_local on the same windows, within
north_star's 1e-5 (test_gpu_ba.close) -- for windows that change from call to call the way a caller's
covisibility windows do: the same camera count again (plan reused), a larger window (capacities
grow), another camera count (a second resident plan), and the structures only the host-built plan
takes (fallback on the same GPU kernels)."""
import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import _abi as A
from lorb_slam_amd import synth
from lorb_slam_amd.runtime import BASolver, LorbError
from test_gpu_ba import close, lm_match

pytestmark = pytest.mark.gpu
OPT10 = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                            parameter_tolerance=0.0)


def check(solver, w, opt, label="", strict=None):
    """one solver call against the oracle: summaries (lm_match), the per-iteration records when the call
    ran on a resident plan (trace_match), the solution to 1e-5.  strict (default: a function tolerance is
    set, so the solve stops before its cost changes reach round-off level): no outcome may differ; at
    tolerance 0 an outcome may differ only where trace_match allows it."""
    if strict is None:
        strict = opt.function_tolerance > 0.0
    Pg, Xg, sg = solver.solve(w, opt)
    gt = solver.trace() if not solver.info()["host_plan_fallback"] else None
    Po, Xo, so, ot = O.ba_local_traced(w, opt)
    flip = lm_match(sg, so, gt=gt, ot=ot if gt is not None else None, label=label)
    assert not strict or flip is None, (label, flip)
    assert close(Pg, Po), np.abs(Pg - Po).max()
    assert close(Xg, Xo), np.abs(Xg - Xo).max()
    return Pg, Xg, sg


def test_solver_c4_reference_order_twice(ctx):
    """C4 window in the reference's camera order, solved twice (the second call with the first
    call's float write-back as its start, as the drop-in's next call sees it): one plan creation,
    band 47 after the RCM relabelling, no host-built fallback.  At tolerance 0 the solve runs into
    cost changes at round-off level (~1e-14 relative by the 10th iteration), where the accept test
    may go either way: the per-iteration records must agree up to there, and an outcome may differ
    only at such an iteration (trace_match)."""
    w0 = synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)
    w, _ = synth.reference_window_order(w0)
    s = BASolver(ctx)
    try:
        P1, X1, _ = check(s, w, OPT10, label="solver c4 ref-order tol0 call 1")
        w2 = dict(w, pose_init=P1.astype(np.float32), point_init=X1.astype(np.float32))
        check(s, w2, OPT10, label="solver c4 ref-order tol0 call 2")
        info = s.info()
        assert info["plan_creations"] == 1 and info["host_plan_fallback"] == 0, info
        assert info["band"] == 47 and info["cholesky"] == 2 and info["reordered"] == 1, info
    finally:
        s.close()


def test_solver_c4_reference_order_ceres_defaults(ctx):
    """the drop-in path (BA::LocalPoseOptimization, src/bundle_adjust.cpp:207-330)
    on the full-size C4 window in the reference's camera order with the options the reference runs
    (Ceres defaults + DENSE_SCHUR, :308-314), twice (the second call from the first's float
    write-back): termination, iterations, accepted steps and every iteration's outcome as the
    oracle's (strict), costs within 1e-10."""
    w0 = synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)
    w, _ = synth.reference_window_order(w0)
    s = BASolver(ctx)
    try:
        P1, X1, s1 = check(s, w, A.LMOptions.default(), label="solver c4 ref-order defaults call 1", strict=True)
        w2 = dict(w, pose_init=P1.astype(np.float32), point_init=X1.astype(np.float32))
        check(s, w2, A.LMOptions.default(), label="solver c4 ref-order defaults call 2", strict=True)
        assert s.info()["plan_creations"] == 1 and s.info()["host_plan_fallback"] == 0
    finally:
        s.close()


def test_solver_windows_that_change(ctx):
    """default Ceres options; camera counts 12 -> 12 (more points: capacities grow) -> 20 -> 12"""
    s = BASolver(ctx)
    try:
        a = synth.ba_window(seed=21, n_kf=12, n_pts=800, n_fixed=2, fixed_obs_per_kf=80)
        b = synth.ba_window(seed=22, n_kf=12, n_pts=3000, n_fixed=3, fixed_obs_per_kf=200)
        c = synth.ba_window(seed=23, n_kf=20, n_pts=1500, n_fixed=1, fixed_obs_per_kf=100)
        for w in (a, b, c, a):
            check(s, w, A.LMOptions.default())
        info = s.info()
        assert info["resident_plans"] == 2 and info["host_plan_fallback"] == 0, info
    finally:
        s.close()


def test_solver_sorted_duplicate(ctx):
    """point-sorted slots (the device build's k_db_sorted path, no counting sort): a camera seen twice
    inside one point's run -- next to the first slot, and at the run's end -- is rejected; the sorted
    window itself solves like the oracle, and the solver stays usable after the errors."""
    s = BASolver(ctx)
    try:
        w0 = synth.ba_window(seed=25, n_kf=12, n_pts=3000, n_fixed=2, fixed_obs_per_kf=150)
        o = np.argsort(np.asarray(w0["obs_point"]), kind="stable")
        uv = np.asarray(w0["obs_uv"]).reshape(-1, 2)
        w = dict(w0, obs_point=np.asarray(w0["obs_point"])[o], obs_frame=np.asarray(w0["obs_frame"])[o], obs_uv=uv[o])
        check(s, w, OPT10)
        opt_slots = np.flatnonzero(np.asarray(w["obs_frame"]) >= 0)
        for k, at in ((int(opt_slots[len(opt_slots) // 2]), 1), (int(opt_slots[len(opt_slots) // 3]), 0)):
            p = w["obs_point"][k]
            run_end = int(np.searchsorted(w["obs_point"], p, side="right"))
            pos = k + 1 if at == 1 else run_end
            dup = dict(w, obs_point=np.insert(w["obs_point"], pos, p), obs_frame=np.insert(w["obs_frame"], pos, w["obs_frame"][k]),
                       obs_uv=np.insert(w["obs_uv"], pos, w["obs_uv"][k], axis=0))
            with pytest.raises(LorbError, match="twice"):
                s.solve(dup, OPT10)
        check(s, w, OPT10)
        assert s.info()["host_plan_fallback"] == 0
    finally:
        s.close()


def test_solver_many_cameras(ctx):
    """the widest device-built window (128 cameras: past the fused covisibility tables' LDS, so
    k_db_cov runs), in caller order and point-sorted, then a 170-camera window, which the device
    build refuses (its camera tables are kernel arguments of <= 128 cameras) and the solver runs on
    a host-built plan -- the same point-major kernels, point groups cut at a 128-camera span; every
    call against the oracle"""
    s = BASolver(ctx)
    try:
        w = synth.ba_window(seed=26, n_kf=128, n_pts=2500, n_fixed=2, fixed_obs_per_kf=40)
        check(s, w, OPT10)
        o = np.argsort(np.asarray(w["obs_point"]), kind="stable")
        uv = np.asarray(w["obs_uv"]).reshape(-1, 2)
        ws = dict(w, obs_point=np.asarray(w["obs_point"])[o], obs_frame=np.asarray(w["obs_frame"])[o], obs_uv=uv[o])
        check(s, ws, OPT10)
        assert s.info()["host_plan_fallback"] == 0
        w170 = synth.ba_window(seed=27, n_kf=170, n_pts=2500, n_fixed=2, fixed_obs_per_kf=40)
        check(s, w170, OPT10)
        assert s.info()["host_plan_fallback"] == 1
        check(s, w, OPT10)
        assert s.info()["host_plan_fallback"] == 0
    finally:
        s.close()


def test_solver_fallback_and_errors(ctx):
    """a point observed twice by one camera (the reference's std::map<Frame*, size_t> cannot hold
    it) is rejected by both plan builders; bad indices are rejected like lorb_ba_local rejects them;
    an empty window runs on the host-built plan; the solver stays usable after every error."""
    s = BASolver(ctx)
    try:
        w = synth.ba_window(seed=24, n_kf=6, n_pts=300, n_fixed=1, fixed_obs_per_kf=40)
        k = int(np.flatnonzero(np.asarray(w["obs_frame"]) >= 0)[0])
        dup = dict(w, obs_point=np.append(w["obs_point"], w["obs_point"][k]),
                   obs_frame=np.append(w["obs_frame"], w["obs_frame"][k]),
                   obs_uv=np.concatenate([np.asarray(w["obs_uv"]).reshape(-1, 2), np.asarray(w["obs_uv"]).reshape(-1, 2)[k:k + 1]]))
        with pytest.raises(LorbError, match="twice"):
            s.solve(dup, OPT10)
        with pytest.raises(LorbError, match="twice"):
            ctx.ba_local([dup], OPT10)
        check(s, w, OPT10)
        assert s.info()["host_plan_fallback"] == 0
        bad = dict(w, obs_frame=np.where(np.arange(len(w["obs_frame"])) == 3, -5, w["obs_frame"]))
        with pytest.raises(LorbError, match="bad frame"):
            s.solve(bad, OPT10)
        bad = dict(w, obs_point=np.where(np.arange(len(w["obs_point"])) == 3, len(w["point_init"]), w["obs_point"]))
        with pytest.raises(LorbError, match="bad point"):
            s.solve(bad, OPT10)
        empty = dict(w, point_init=np.zeros((0, 3), np.float32), obs_point=np.zeros(0, np.int32),
                     obs_frame=np.zeros(0, np.int32), obs_uv=np.zeros((0, 2), np.float32))
        P, X, sm = s.solve(empty, OPT10)
        assert P.shape == (6, 6) and X.shape == (0, 3) and s.info()["host_plan_fallback"] == 1
        check(s, w, OPT10)  # still usable after the errors
    finally:
        s.close()


def wide_window(seed, n_kf, n_pts, obs_len, n_fixed=2, fixed_obs=60, fx=435.2, fy=435.2, cx=367.5, cy=252.2):
    """a long straight window (camera i at (0.1 i, 0, 0), no rotation: every point in front of every
    camera), each point seen by obs_len consecutive keyframes, and point 0 by ALL of them"""
    rng = np.random.default_rng(seed)
    C = np.stack([0.1 * np.arange(-n_fixed, n_kf), np.zeros(n_kf + n_fixed), np.zeros(n_kf + n_fixed)], 1)
    poses = np.concatenate([np.zeros((n_kf + n_fixed, 3)), -C], 1)  # rows: fixed -n_fixed..-1, then window
    pts = np.stack([rng.uniform(-6, 0.1 * n_kf + 6, n_pts), rng.uniform(-3, 3, n_pts), rng.uniform(4, 20, n_pts)], 1)
    obs_p, obs_f = [], []
    for q in range(n_pts):
        fr = range(n_kf) if q == 0 else range(s0 := int(rng.integers(0, n_kf - obs_len + 1)), s0 + obs_len)
        for f in fr:
            obs_p.append(q); obs_f.append(f)
    for j in range(n_fixed):
        for q in np.sort(rng.choice(np.arange(1, n_pts), size=fixed_obs, replace=False)):
            obs_p.append(q); obs_f.append(-1 - j)
    obs_p = np.asarray(obs_p, np.int32); obs_f = np.asarray(obs_f, np.int32)
    row = np.where(obs_f >= 0, n_fixed + obs_f, n_fixed - 1 - (-1 - obs_f))
    Xc = pts[obs_p] + poses[row, 3:]
    uv = np.stack([fx * Xc[:, 0] / Xc[:, 2] + cx, fy * Xc[:, 1] / Xc[:, 2] + cy], 1) + rng.normal(0, 0.5, (len(obs_p), 2))
    pose_init = poses[n_fixed:].copy()
    pose_init[:, :3] += rng.normal(0, 2e-3, (n_kf, 3))
    pose_init[:, 3:] += rng.normal(0, 2e-2, (n_kf, 3))
    return dict(pose_init=pose_init.astype(np.float32), fixed_pose=poses[n_fixed - 1::-1].astype(np.float32).reshape(-1, 6),
                point_init=(pts + rng.normal(0, 5e-2, pts.shape)).astype(np.float32), obs_point=obs_p, obs_frame=obs_f,
                obs_uv=uv.astype(np.float32), intr=(np.float32(fx), np.float32(fy), np.float32(cx), np.float32(cy)))


def test_solver_kgb_fallback_between_normal_windows(ctx):
    """a resident plan, then a window with one point observed by 260 cameras (>= kGB = 256
    observations, cameras 259 apart: a point group holds neither, so both plan builders refuse it
    with LORB_E_UNSUPPORTED -- DESIGN §7), then the first window again on its resident plan: the
    failed builds leave no stale plan or scratch behind, every result against the oracle"""
    opt = A.LMOptions.default(max_num_iterations=3, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    s = BASolver(ctx)
    try:
        a = synth.ba_window(seed=31, n_kf=12, n_pts=900, n_fixed=2, fixed_obs_per_kf=90)
        check(s, a, opt)
        big = wide_window(seed=32, n_kf=260, n_pts=1200, obs_len=3)
        assert int(np.sum(np.asarray(big["obs_point"]) == 0)) == 260
        with pytest.raises(LorbError, match="observations"):
            s.solve(big, opt)
        check(s, a, opt)
        info = s.info()
        assert info["host_plan_fallback"] == 0 and info["plan_creations"] == 1, info
    finally:
        s.close()


def test_solver_lru_eviction(ctx):
    """six camera counts through the four resident plans (least recently used evicted), then the
    evicted counts again: every call against the oracle"""
    s = BASolver(ctx)
    try:
        wins = [synth.ba_window(seed=40 + k, n_kf=k, n_pts=80 * k, n_fixed=1, fixed_obs_per_kf=30) for k in range(6, 12)]
        # default Ceres tolerances: at tolerance 0 these small windows converge to machine precision
        # and the stopping iteration is rounding-determined
        for w in wins + wins[:2]:
            check(s, w, A.LMOptions.default())
        info = s.info()
        assert info["resident_plans"] == 4 and info["plan_creations"] == 8 and info["host_plan_fallback"] == 0, info
    finally:
        s.close()
