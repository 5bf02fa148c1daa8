"""GPU parity: bundle adjustment (liblorb.so) vs the oracle's Ceres-LM restatement.

Tolerance (north_star): poses / points within 1e-5 relative.  Relative is taken per block
against max(|oracle|, 1) for angle-axis / translation / point coordinates, i.e.
|gpu - oracle| <= 1e-5 * max(|oracle|, 1)."""
import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import _abi as A
from lorb_slam_amd import synth

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(b), 1.0))


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def trace_match(gt, ot, cost_rtol=1e-10, strict_to=1e-12, flip_at=1e-13, label=""):
    """Iteration-level LM parity: the GPU's per-iteration records (lorb_ba_plan_trace)
    against the oracle's (or_lm_trace).  Iteration by iteration: the cost at the current point and the
    candidate's cost within cost_rtol relative, the model cost change within cost_rtol of the cost, the
    radius within 1e-6 relative (it compounds the step-quality ratio), and the same outcome (accepted /
    rejected / invalid / tolerance stop) -- up to and including the first iteration whose relative cost
    change |cost - new_cost| / cost is at most strict_to.  From there on the accept test compares cost
    changes at the level of the round-off of two different summation orders (reduction trees, Cholesky
    order), and the two solves may part: an outcome may then differ, but only at an iteration whose
    relative cost change is at most flip_at (in either trace).  Returns the index of the first differing
    outcome (None: every outcome agrees and the traces have the same length)."""
    worst = dict(cost=0.0, new_cost=0.0, radius=0.0, mcc_over_cost=0.0)
    tail = None  # index of the first round-off-level iteration
    for i, (g, o) in enumerate(zip(gt, ot)):
        assert g["iteration"] == o["iteration"] == i + 1, (i, g, o)
        rc_o = abs(o["cost"] - o["new_cost"]) / abs(o["cost"])
        rc_g = abs(g["cost"] - g["new_cost"]) / abs(g["cost"])
        if tail is not None:  # past the strict part: only where an outcome parts is checked
            if g["outcome"] != o["outcome"]:
                assert min(rc_o, rc_g) <= flip_at, (label, i, rc_o, rc_g, g, o)
                print(f"{label}: outcomes agree through iteration {tail + 1} (relative cost change there "
                      f"{abs(ot[tail]['cost'] - ot[tail]['new_cost']) / ot[tail]['cost']:.2e}); they part at iteration "
                      f"{i + 1}: {g['outcome']} (gpu) vs {o['outcome']} (oracle), relative cost change {rc_o:.2e} / "
                      f"{rc_g:.2e}; max differences before {worst}")
                return i
            continue
        assert _rel(g["cost"], o["cost"]) <= cost_rtol, (label, i, g, o)
        if g["outcome"] != o["outcome"]:  # the first round-off-level iteration may already part
            assert min(rc_o, rc_g) <= flip_at, (label, i, rc_o, rc_g, g, o)
            print(f"{label}: outcomes agree through iteration {i}; they part at iteration {i + 1}: "
                  f"{g['outcome']} (gpu) vs {o['outcome']} (oracle), relative cost change {rc_o:.2e} / {rc_g:.2e}; "
                  f"max differences before {worst}")
            return i
        assert abs(g["model_cost_change"] - o["model_cost_change"]) <= cost_rtol * abs(o["cost"]), (label, i, g, o)
        assert _rel(g["radius"], o["radius"]) <= 1e-6, (label, i, g, o)
        if o["outcome"] != "invalid":
            assert _rel(g["new_cost"], o["new_cost"]) <= cost_rtol, (label, i, g, o)
            worst["new_cost"] = max(worst["new_cost"], _rel(g["new_cost"], o["new_cost"]))
        worst["cost"] = max(worst["cost"], _rel(g["cost"], o["cost"]))
        worst["radius"] = max(worst["radius"], _rel(g["radius"], o["radius"]))
        worst["mcc_over_cost"] = max(worst["mcc_over_cost"], abs(g["model_cost_change"] - o["model_cost_change"]) / abs(o["cost"]))
        if rc_o <= strict_to:
            tail = i
    if tail is None:
        assert len(gt) == len(ot), (label, len(gt), len(ot))
        print(f"{label}: {len(gt)} iterations, identical outcomes; max relative differences {worst}")
    else:
        print(f"{label}: identical outcomes through all {min(len(gt), len(ot))} iterations (strict through "
              f"{tail + 1}); max relative differences {worst}")
    return None


def lm_match(g, o, cost_rtol=1e-8, gt=None, ot=None, label=""):
    """The LM summaries agree to the north_star contract: same iteration count, same count of
    accepted steps, final cost within cost_rtol relative.  With the per-iteration records (gt, ot) the
    traces are compared too (trace_match); a differing accepted-step count is then allowed only when
    the traces show the outcomes parting at a round-off-level cost change (the solution itself is
    checked to 1e-5 by the caller).  The same holds for the iteration count: at tolerance 0 a solve
    may stop on an exactly-zero cost change (function tolerance 0), which one summation order reaches
    and the other does not -- allowed only behind such a round-off-level parting."""
    assert abs(g["final_cost"] - o["final_cost"]) <= cost_rtol * abs(o["final_cost"]), (g, o)
    flip = trace_match(gt, ot, label=label) if gt is not None else None
    if g["iterations"] != o["iterations"]:
        assert flip is not None, (g, o)
        print(f"{label}: iterations gpu {g['iterations']} vs oracle {o['iterations']} after the round-off "
              f"parting at iteration {flip + 1}")
    if g["successful_steps"] != o["successful_steps"]:
        assert flip is not None, (g, o)
        print(f"{label}: accepted steps gpu {g['successful_steps']} vs oracle {o['successful_steps']} after the "
              f"round-off flip at iteration {flip + 1}")
    return flip


@pytest.mark.parametrize("quirk", [True, False])
def test_pose_only_default_options(ctx, quirk):
    pb = synth.pose_only_batch(seed=1, n_frames=16, n_res=200, quirk=quirk)
    pg, Tg, sg = ctx.ba_pose_only(pb)
    po, To, so = O.ba_pose_only(pb)
    assert close(pg, po), np.abs(pg - po).max()
    assert np.allclose(Tg, To, rtol=1e-5, atol=1e-6)
    for a, b in zip(sg, so):
        assert a["termination"] == b["termination"] and a["iterations"] == b["iterations"]
        assert a["successful_steps"] == b["successful_steps"], (a, b)
        assert abs(a["final_cost"] - b["final_cost"]) <= 1e-6 * b["final_cost"]


def test_pose_only_fixed_iterations_and_edge(ctx):
    pb = synth.pose_only_batch(seed=4, n_frames=5, n_res=1500)
    # frame with zero residuals (empty ceres::Problem leaves the pose untouched)
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    pg, _, sg = ctx.ba_pose_only(pb, opt)
    po, _, so = O.ba_pose_only(pb, opt)
    # at tolerance 0 the solve runs into machine-precision convergence, where the stopping
    # iteration (exact-zero cost change / non-positive model decrease) is rounding-determined:
    # compare the solution only
    assert close(pg, po), np.abs(pg - po).max()
    empty = dict(res_off=np.array([0, 0], np.int32), intr=pb["intr"][:1], pose_init=pb["pose_init"][:1],
                 pts3d=np.zeros((0, 3), np.float32), obs2d=np.zeros((0, 2), np.float32))
    pg, _, _ = ctx.ba_pose_only(empty)
    assert np.array_equal(pg[0], pb["pose_init"][0].astype(np.float64))


def test_pose_only_identity_init_small_angle_branch(ctx):
    pb = synth.pose_only_batch(seed=9, n_frames=3, n_res=300)
    pb["pose_init"][:, :3] = 0.0  # theta^2 <= eps: first-order AngleAxisRotatePoint branch
    pg, _, _ = ctx.ba_pose_only(pb)
    po, _, _ = O.ba_pose_only(pb)
    assert close(pg, po), np.abs(pg - po).max()


@pytest.mark.parametrize("n_kf,n_pts,n_fixed", [(6, 300, 2), (20, 4000, 2)])
def test_local_ba_default_options(ctx, n_kf, n_pts, n_fixed):
    w = synth.ba_window(seed=3, n_kf=n_kf, n_pts=n_pts, n_fixed=n_fixed, fixed_obs_per_kf=max(60, n_pts // 10))
    Pg, Xg, sg = ctx.ba_local([w])
    Po, Xo, so = O.ba_local([w])
    assert sg[0]["termination"] == so[0]["termination"], (sg, so)
    assert sg[0]["iterations"] == so[0]["iterations"], (sg, so)
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()
    assert abs(sg[0]["final_cost"] - so[0]["final_cost"]) <= 1e-8 * so[0]["final_cost"]


def test_local_ba_c3_ten_iterations(ctx):
    """BASELINE config 2 shape: 20 KF / 4k points / 30k obs (+2 fixed KFs), exactly 10 LM its."""
    w = synth.ba_window(seed=3, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)
    assert len(w["obs_point"]) == 30000 + 800
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    Pg, Xg, sg, gt = plan_traced(ctx, w, opt)
    Po, Xo, so, ot = O.ba_local_traced(w, opt)
    assert sg["iterations"] == so["iterations"] == 10 and len(gt) == 10
    lm_match(sg, so, gt=gt, ot=ot, label="c3 tol0")
    assert close(Pg, Po), np.abs(Pg - Po).max()
    assert close(Xg, Xo), np.abs(Xg - Xo).max()


@pytest.mark.parametrize("n_kf,obs_lens", [(20, (7, 8)), (40, (2, 30)), (100, (7, 8))])
def test_local_ba_point_order_without_camera_locality(ctx, n_kf, obs_lens):
    """Points in draw order (no camera locality: a point group's camera window spans most of the
    window) and, second case, points seen by 2 or 30 keyframes (a camera band of 29): the
    point-major path's group windows are wide and its partials sparse -- the result must not depend
    on the point order's locality, only its speed does.  The 100-camera case gives group windows
    wider than 64 cameras (k_ba_ls's two-word camera masks)."""
    w = synth.ba_window(seed=17, n_kf=n_kf, n_pts=2000, n_fixed=2, fixed_obs_per_kf=200, obs_lens=obs_lens,
                        point_order="random")
    opt = A.LMOptions.default(max_num_iterations=8, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    Pg, Xg, sg = ctx.ba_local([w], opt)
    Po, Xo, so = O.ba_local([w], opt)
    lm_match(sg[0], so[0])
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()


@pytest.mark.parametrize("n_kf,n_pts,n_fixed,pm", [(70, 3000, 2, 1), (100, 5000, 2, 1), (128, 6000, 3, 1),
                                                   (20, 4000, 2, 1), (50, 10000, 5, 1)])
def test_local_ba_schur_path_by_window(ctx, n_kf, n_pts, n_fixed, pm):
    """The Schur path each window shape takes, and its parity: every window runs the point-major path
    (k_ba_ls / k_ba_red / k_ba_bs2; camera masks of two words: windows of up to 128 cameras), C3 with
    1024-thread partial reductions (<= 256 blocks), C4 with 512 (372 blocks)."""
    from lorb_slam_amd.runtime import BAPlan
    w = synth.ba_window(seed=29, n_kf=n_kf, n_pts=n_pts, n_fixed=n_fixed, fixed_obs_per_kf=100)
    opt = A.LMOptions.default(max_num_iterations=6, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    plan = BAPlan(ctx, [w])
    try:
        info = plan.info()
        assert info["point_major"] == pm, info
        if pm:
            assert info["red_threads"] == (1024 if info["blocks"] <= 256 else 512 if info["blocks"] <= 1024 else 256), info
    finally:
        plan.close()
    Pg, Xg, sg = ctx.ba_local([w], opt)
    Po, Xo, so = O.ba_local([w], opt)
    lm_match(sg[0], so[0])
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()


@pytest.mark.parametrize("order", ["first_kf", "random"])
def test_local_ba_window_over_128_cameras(ctx, order):
    """A 150-camera window (host-built plan): point groups are cut where a group's camera window
    would pass 128 cameras (k_ba_ls's two-word masks; with random point order that cuts most groups
    early), and the solve still matches the oracle."""
    from lorb_slam_amd.runtime import BAPlan
    w = synth.ba_window(seed=41, n_kf=150, n_pts=4000, n_fixed=2, fixed_obs_per_kf=100, point_order=order)
    opt = A.LMOptions.default(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    plan = BAPlan(ctx, [w])
    try:
        info = plan.info()
        assert info["cameras"] == 150 and info["point_major"] == 1, info
        if order == "random":  # groups end at the span limit long before 256 observations
            assert info["point_groups"] > len(w["obs_point"]) // 256 + 1, info
    finally:
        plan.close()
    Pg, Xg, sg = ctx.ba_local([w], opt)
    Po, Xo, so = O.ba_local([w], opt)
    lm_match(sg[0], so[0])
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()


def test_local_ba_plan_limits(ctx):
    """What the point-major path refuses, loudly (LORB_E_UNSUPPORTED): a point whose cameras lie more
    than 127 apart in every camera order (seen by all 140 cameras) in a host-built plan, and a
    device-built plan of more than 128 cameras (the drop-in solver falls back to a host-built plan
    for it, lorb_ba_solver.hip)."""
    from lorb_slam_amd.runtime import BAPlan, BAPlanDev, LorbError
    w = synth.ba_window(seed=42, n_kf=140, n_pts=300, n_fixed=1, fixed_obs_per_kf=20, obs_lens=(140, 7))
    with pytest.raises(LorbError, match="apart"):
        BAPlan(ctx, [w])
    w2 = synth.ba_window(seed=43, n_kf=130, n_pts=2000, n_fixed=1, fixed_obs_per_kf=50)
    arrays = BAPlanDev.upload(ctx, w2)
    try:
        with pytest.raises(LorbError, match="128 cameras"):
            BAPlanDev(ctx, arrays, 130, 1, w2["intr"])
    finally:
        for a in arrays.values():
            a.free()


def test_local_ba_batched_ragged_windows(ctx):
    wins = [synth.ba_window(seed=10 + i, n_kf=k, n_pts=p, n_fixed=nf, fixed_obs_per_kf=50)
            for i, (k, p, nf) in enumerate([(3, 100, 1), (8, 700, 2), (12, 900, 3), (5, 257, 1)])]
    # an unobserved point and an empty window
    wins[1]["point_init"] = np.concatenate([wins[1]["point_init"], [[1.0, 2.0, 9.0]]]).astype(np.float32)
    empty = dict(pose_init=np.zeros((2, 6), np.float32), fixed_pose=np.zeros((0, 6), np.float32),
                 point_init=np.zeros((3, 3), np.float32), obs_point=np.zeros(0, np.int32),
                 obs_frame=np.zeros(0, np.int32), obs_uv=np.zeros((0, 2), np.float32), intr=wins[0]["intr"])
    wins.append(empty)
    Pg, Xg, sg = ctx.ba_local(wins)
    Po, Xo, so = O.ba_local(wins)
    for i in range(len(wins)):
        assert close(Pg[i], Po[i]), (i, np.abs(Pg[i] - Po[i]).max())
        assert close(Xg[i], Xo[i]), (i, np.abs(Xg[i] - Xo[i]).max())
    assert np.array_equal(Xg[1][-1], np.array([1.0, 2.0, 9.0]))
    assert np.array_equal(Pg[-1], np.zeros((2, 6)))


def test_plan_resolve_is_repeatable(ctx):
    from lorb_slam_amd.runtime import BAPlan
    w = synth.ba_window(seed=5, n_kf=10, n_pts=1000, n_fixed=2, fixed_obs_per_kf=100)
    plan = BAPlan(ctx, [w])
    plan.solve(); a = plan.read()
    plan.solve(); b = plan.read()
    assert np.array_equal(a[0][0], b[0][0]) and np.array_equal(a[1][0], b[1][0])
    plan.close()


@pytest.mark.parametrize("n_kf,n_pts", [(10, 300), (30, 400), (54, 300)])
def test_local_ba_dense_covisibility(ctx, n_kf, n_pts):
    """Every point seen by every window KF: S is fully dense (band = n-1).  Covers the
    multi-row-per-lane register panel and the global-memory (band > LDS) Cholesky path."""
    w = synth.ba_window(seed=21, n_kf=n_kf, n_pts=n_pts, n_fixed=1, fixed_obs_per_kf=50, obs_lens=(n_kf,))
    opt = A.LMOptions.default(max_num_iterations=6)
    Pg, Xg, sg = ctx.ba_local([w], opt)
    Po, Xo, so = O.ba_local([w], opt)
    assert sg[0]["iterations"] == so[0]["iterations"]
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()


@pytest.mark.parametrize("obs_len,kind", [(2, 1), (3, 2), (8, 2)])
def test_local_ba_narrow_band(ctx, obs_len, kind):
    """Points seen by obs_len consecutive KFs: band 6*obs_len - 1 (11, 17, 47).  The two-sided
    Cholesky's back-substitution needs the full inverse of each 16 x 16 diagonal block, which the
    band holds only for bw >= 15, so a band of 11 takes k_ba_chol_w (kind 1)."""
    from lorb_slam_amd.runtime import BAPlan
    w = synth.ba_window(seed=23, n_kf=30, n_pts=1500, n_fixed=2, fixed_obs_per_kf=100, obs_lens=(obs_len,))
    opt = A.LMOptions.default(max_num_iterations=8, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    plan = BAPlan(ctx, [w])
    plan.solve(opt)
    (Pg,), (Xg,), (sg,) = plan.read()
    info = plan.info()
    plan.close()
    Po, Xo, so = O.ba_local([w], opt)
    assert info["band"] == 6 * obs_len - 1 and info["cholesky"] == kind, info
    assert sg["iterations"] == so[0]["iterations"]
    lm_match(sg, so[0])
    assert close(Pg, Po[0]), np.abs(Pg - Po[0]).max()
    assert close(Xg, Xo[0]), np.abs(Xg - Xo[0]).max()


def plan_traced(ctx, w, opt):
    """solve one window on a host-built plan: poses, points, summary and the per-iteration records"""
    from lorb_slam_amd.runtime import BAPlan
    plan = BAPlan(ctx, [w])
    try:
        plan.solve(opt)
        (Pg,), (Xg,), (sg,) = plan.read()
        return Pg, Xg, sg, plan.trace(0)
    finally:
        plan.close()


def test_local_ba_c4_full_size(ctx):
    """BASELINE config 3 (the bench workload): 50 KF / 10k points / 77k obs (+5 fixed KFs), 10 LM its,
    at full size against the oracle, iteration by iteration."""
    w = synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)
    assert len(w["obs_point"]) == 77000
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    Pg, Xg, sg, gt = plan_traced(ctx, w, opt)
    Po, Xo, so, ot = O.ba_local_traced(w, opt)
    assert sg["iterations"] == so["iterations"] == 10 and len(gt) == 10
    lm_match(sg, so, gt=gt, ot=ot, label="c4 tol0")
    assert close(Pg, Po), np.abs(Pg - Po).max()
    assert close(Xg, Xo), np.abs(Xg - Xo).max()


@pytest.mark.parametrize("size", ["c3", "c4"])
def test_local_ba_ceres_default_options_full_size(ctx, size):
    """BA::LocalPoseOptimization's real options -- Ceres defaults with DENSE_SCHUR
    (50 iterations, function_tolerance 1e-6, gradient 1e-10, parameter 1e-8;
    src/bundle_adjust.cpp:308-314) -- on the full-size C3 and C4 windows.  The termination the drop-in
    decides must be the oracle's: same termination, iterations and accepted steps (strict), and the
    per-iteration records identical in outcome with costs within 1e-10."""
    kw = dict(seed=3, n_kf=20, n_pts=4000, n_fixed=2) if size == "c3" else dict(seed=4, n_kf=50, n_pts=10000, n_fixed=5)
    w = synth.ba_window(fixed_obs_per_kf=400, **kw)
    opt = A.LMOptions.default()
    Pg, Xg, sg, gt = plan_traced(ctx, w, opt)
    Po, Xo, so, ot = O.ba_local_traced(w, opt)
    assert sg["termination"] == so["termination"], (sg, so)
    assert sg["successful_steps"] == so["successful_steps"], (sg, so)
    assert lm_match(sg, so, gt=gt, ot=ot, label=f"{size} ceres defaults") is None
    assert close(Pg, Po), np.abs(Pg - Po).max()
    assert close(Xg, Xo), np.abs(Xg - Xo).max()


@pytest.mark.parametrize("size", ["c3", "c4"])
def test_local_ba_reference_camera_order(ctx, size):
    """the window in the order BA::LocalPoseOptimization builds it ([curr] +
    covisible frames by ascending weight, src/bundle_adjust.cpp:210-220) scatters S's blocks; the plan
    reorders the cameras (reverse Cuthill-McKee), keeps the banded two-sided Cholesky (band 47) and
    returns the poses in the caller's order, within 1e-5 of the oracle on the same window."""
    from lorb_slam_amd.runtime import BAPlan
    n_kf, n_pts, nf, fo, seed = (20, 4000, 2, 400, 3) if size == "c3" else (50, 10000, 5, 400, 4)
    w0 = synth.ba_window(seed=seed, n_kf=n_kf, n_pts=n_pts, n_fixed=nf, fixed_obs_per_kf=fo)
    w, order = synth.reference_window_order(w0)
    assert not np.array_equal(order, np.arange(n_kf))
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    plan = BAPlan(ctx, [w])
    plan.solve(opt)
    Pg, Xg, sg = plan.read()
    info = plan.info()
    plan.close()
    assert info["reordered"] == 1 and info["band"] == 47 and info["cholesky"] == 2, info
    Po, Xo, so = O.ba_local([w], opt)
    lm_match(sg[0], so[0])
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()
    # the same window in temporal order gives the same solution (up to the elimination order)
    Pt, Xt, _ = ctx.ba_local([w0], opt)
    assert close(Pg[0], Pt[0][order]) and close(Xg[0], Xt[0])


@pytest.mark.parametrize("shape", ["c4", "c3"])
def test_local_ba_eight_c4_windows_independent(ctx, shape):
    """BASELINE config 4 shape on one GPU: 8 C4 windows in one plan.  Size-independent property:
    batching never couples windows -- each window's result is bit-identical to its solo solve.  The
    C3 case also crosses reduction widths (solo: 1024-thread k_ba_red, batched: 256), whose group
    sums use the same fixed subsets and order."""
    kw = dict(n_kf=50, n_pts=10000, n_fixed=5) if shape == "c4" else dict(n_kf=20, n_pts=4000, n_fixed=2)
    wins = [synth.ba_window(seed=40 + i, fixed_obs_per_kf=400, **kw) for i in range(8)]
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    if shape == "c3":
        from lorb_slam_amd.runtime import BAPlan
        solo, batch = BAPlan(ctx, wins[:1]), BAPlan(ctx, wins)
        assert solo.info()["red_threads"] == 1024 and batch.info()["red_threads"] < 1024
        solo.close(); batch.close()
    Pb, Xb, sb = ctx.ba_local(wins, opt)
    for i in (0, 5):
        Ps, Xs, ss = ctx.ba_local([wins[i]], opt)
        assert np.array_equal(Pb[i], Ps[0]) and np.array_equal(Xb[i], Xs[0])
        assert sb[i]["final_cost"] == ss[0]["final_cost"]


def test_plan_group_bit_identical(ctx):
    """lorb_ba_group: separately built plans solved by one set of launches.  Members: a plan of two
    C4 windows, a plan of one C3 window and a plan of one C4 window.  Each window's poses, points,
    summary and LM trace equal those of its own plan solved alone, bit for bit; the group ran fused
    and replays its graph (one capture for two solves)."""
    from lorb_slam_amd.runtime import BAGroup, BAPlan
    c4 = [synth.ba_window(seed=40 + i, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400) for i in range(3)]
    c3 = synth.ba_window(seed=7, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    members = [c4[:2], [c3], c4[2:]]
    gp = [BAPlan(ctx, m) for m in members]
    sp = [BAPlan(ctx, m) for m in members]
    G = BAGroup(ctx, gp)
    try:
        for rep in range(2):
            G.solve(opt)
            for p in sp:
                p.solve(opt)
            for a, b in zip(gp, sp):
                ra, rb = a.read(), b.read()
                for w in range(len(ra[0])):
                    assert np.array_equal(ra[0][w], rb[0][w]) and np.array_equal(ra[1][w], rb[1][w]), (rep, w)
                    assert ra[2][w] == rb[2][w], (rep, w)
                    assert a.trace(w) == b.trace(w), (rep, w)
        assert G.info() == {"plans": 3, "fused_solves": 2, "captures": 1}, G.info()
    finally:
        G.close()
        for p in gp + sp:
            p.close()


def test_plan_group_members_stop_at_different_iterations(ctx):
    """Ceres-default options (tolerances on, 50 iterations): the group's members terminate at different
    iterations (a converged window early-exits every later launch while the others go on); each one
    still equals its own solve bit for bit, termination and trace included, and the oracle's summary."""
    from lorb_slam_amd.runtime import BAGroup, BAPlan
    wins = [synth.ba_window(seed=7, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400),
            synth.ba_window(seed=41, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400),
            synth.ba_window(seed=8, n_kf=24, n_pts=3000, n_fixed=2, fixed_obs_per_kf=300)]
    opt = A.LMOptions.default()
    gp = [BAPlan(ctx, [w]) for w in wins]
    sp = [BAPlan(ctx, [w]) for w in wins]
    G = BAGroup(ctx, gp)
    try:
        G.solve(opt)
        for p in sp:
            p.solve(opt)
        its = []
        for i, (a, b) in enumerate(zip(gp, sp)):
            ra, rb = a.read(), b.read()
            assert np.array_equal(ra[0][0], rb[0][0]) and np.array_equal(ra[1][0], rb[1][0]), i
            assert ra[2][0] == rb[2][0], (i, ra[2][0], rb[2][0])
            assert a.trace(0) == b.trace(0), i
            its.append(ra[2][0]["iterations"])
            _, _, so, ot = O.ba_local_traced(wins[i], opt)
            lm_match(ra[2][0], so, gt=a.trace(0), ot=ot, label=f"group member {i}")
        assert G.info()["fused_solves"] == 1, G.info()
        assert len(set(its)) > 1, its  # the members did stop at different iterations
    finally:
        G.close()
        for p in gp + sp:
            p.close()


@pytest.mark.parametrize("f", [2, 5])
def test_local_ba_partial_runs(ctx, f, monkeypatch):
    """partial runs -- f consecutive point groups per k_ba_ls_sup workgroup, their
    camera-block sums added into ONE partial (the path of windows with more than 512 point groups;
    LORB_SG_F forces it here on C4 / C3 windows).  Oracle parity iteration by iteration, poses and
    points within 1e-5; a window batched with another equals its solo solve bit for bit; the
    device-built plan takes the same path."""
    from lorb_slam_amd.runtime import BAPlan, BAPlanDev
    monkeypatch.setenv("LORB_SG_F", str(f))
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    w = synth.ba_window(seed=40, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)
    w3 = synth.ba_window(seed=3, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)
    plan = BAPlan(ctx, [w])
    try:
        plan.solve(opt)
        (Pg,), (Xg,), (sg,) = plan.read()
        gt, info = plan.trace(0), plan.info()
    finally:
        plan.close()
    assert info["partial_runs"] == (info["point_groups"] + f - 1) // f, info
    Po, Xo, so, ot = O.ba_local_traced(w, opt)
    lm_match(sg, so, gt=gt, ot=ot, label=f"partial runs of {f}")
    assert close(Pg, Po), np.abs(Pg - Po).max()
    assert close(Xg, Xo), np.abs(Xg - Xo).max()
    Pb, Xb, sb = ctx.ba_local([w3, w], opt)
    Ps, Xs, ss = ctx.ba_local([w], opt)
    assert np.array_equal(Pb[1], Ps[0]) and np.array_equal(Xb[1], Xs[0]) and sb[1] == ss[0]
    arrays, order = _dev_window(ctx, w3)
    dplan = BAPlanDev(ctx, arrays, len(w3["pose_init"]), len(w3["fixed_pose"]), w3["intr"])
    try:
        dplan.solve(opt)
        Pd, Xd, sd = dplan.read()
        dinfo = dplan.info()
    finally:
        dplan.close()
        for a in arrays.values():
            a.free()
    assert dinfo["partial_runs"] == (dinfo["point_groups"] + f - 1) // f, dinfo
    Po3, Xo3, so3 = O.ba_local([w3], opt)
    lm_match(sd[0], so3[0])
    assert close(Pd[0], Po3[0]) and close(Xd[0], Xo3[0])


def _dev_window(ctx, w, extra_pts=37, extra_obs=500, shuffle_seed=None, holes=0):
    """Upload window w into device arrays with spare capacity, optionally with the observations in
    a shuffled slot order and `holes` unused slots (frame < -n_fixed) spread among them."""
    rng = np.random.default_rng(shuffle_seed or 0)
    K = len(w["obs_point"])
    op, of, uv = w["obs_point"].copy(), w["obs_frame"].copy(), w["obs_uv"].copy()
    order = rng.permutation(K) if shuffle_seed is not None else np.arange(K)
    op, of, uv = op[order], of[order], uv[order]
    if holes:
        at = np.sort(rng.choice(K + holes, size=holes, replace=False))
        keep = np.setdiff1d(np.arange(K + holes), at)
        op2 = np.zeros(K + holes, np.int32); of2 = np.full(K + holes, -10 ** 6, np.int32); uv2 = np.zeros((K + holes, 2), np.float32)
        op2[keep], of2[keep], uv2[keep] = op, of, uv
        op2[at] = rng.integers(0, 10 ** 6, holes)  # garbage point ids in unused slots are ignored
        op, of, uv = op2, of2, uv2
    Kc, P = len(op) + extra_obs, len(w["point_init"])
    pad = lambda a, n, fill=0: np.concatenate([a, np.full((n - len(a),) + a.shape[1:], fill, a.dtype)])
    arrays = dict(n_points=ctx.to_device(np.array([P], np.int32)), n_obs=ctx.to_device(np.array([len(op)], np.int32)),
                  pose_init=ctx.to_device(w["pose_init"].astype(np.float32)),
                  fixed_pose=ctx.to_device(w["fixed_pose"].astype(np.float32).reshape(-1, 6)),
                  point_init=ctx.to_device(pad(w["point_init"].astype(np.float32), P + extra_pts)),
                  obs_point=ctx.to_device(pad(op.astype(np.int32), Kc)), obs_frame=ctx.to_device(pad(of.astype(np.int32), Kc)),
                  obs_uv=ctx.to_device(pad(uv.astype(np.float32), Kc)))
    return arrays, order


@pytest.mark.parametrize("case", ["c3_sorted", "c3_shuffled_holes", "c4_reference_order", "small_ragged"])
def test_device_built_plan(ctx, case):
    """the plan built on the device from HBM-resident observation arrays (point
    sort, covisibility, camera order, groups, Schur pair lists) solves to the oracle's solution
    within 1e-5; unused slots and slot order do not matter beyond round-off."""
    from lorb_slam_amd.runtime import BAPlanDev
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
    if case.startswith("c3"):
        w = synth.ba_window(seed=3, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)
    elif case == "c4_reference_order":
        w, _ = synth.reference_window_order(synth.ba_window(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400))
    else:
        w = synth.ba_window(seed=12, n_kf=7, n_pts=500, n_fixed=2, fixed_obs_per_kf=50)
    arrays, order = _dev_window(ctx, w, shuffle_seed=5 if "shuffled" in case else None, holes=700 if "holes" in case else 0)
    plan = BAPlanDev(ctx, arrays, len(w["pose_init"]), len(w["fixed_pose"]), w["intr"])
    plan.solve(opt)
    Pg, Xg, sg = plan.read()
    info = plan.info()
    # the oracle on the same observations in the same per-point order (stable sort by point)
    srt = np.argsort(w["obs_point"][order], kind="stable")
    wo = dict(w, obs_point=w["obs_point"][order][srt], obs_frame=w["obs_frame"][order][srt], obs_uv=w["obs_uv"][order][srt])
    Po, Xo, so = O.ba_local([wo], opt)
    plan.close()
    for a in arrays.values():
        a.free()
    assert info["observations"] == len(w["obs_point"]) and info["points"] == len(w["point_init"])
    if case != "small_ragged":
        assert info["band"] == 47 and info["cholesky"] == 2, info
    lm_match(sg[0], so[0])
    assert close(Pg[0], Po[0]), np.abs(Pg[0] - Po[0]).max()
    assert close(Xg[0], Xo[0]), np.abs(Xg[0] - Xo[0]).max()


def test_device_built_plan_update_and_result(ctx):
    """The same plan object rebuilt for a changed window (more observations, a keyframe's slots
    marked unused) equals a fresh host plan; result_dev writes float poses in the caller's order."""
    from lorb_slam_amd.runtime import BAPlanDev
    opt = A.LMOptions.default(max_num_iterations=6)
    w = synth.ba_window(seed=31, n_kf=10, n_pts=1200, n_fixed=2, fixed_obs_per_kf=100)
    arrays, _ = _dev_window(ctx, w, extra_obs=3000)
    plan = BAPlanDev(ctx, arrays, 10, 2, w["intr"])
    plan.solve(opt)
    # drop keyframe 0's observations (slots unused) and rebuild in place
    of = w["obs_frame"].copy()
    of[of == 0] = -10 ** 6
    K = len(of)
    buf = np.full(arrays["obs_frame"].shape[0], 0, np.int32); buf[:K] = of
    arrays["obs_frame"].free(); arrays["obs_frame"] = ctx.to_device(buf)
    plan.update(arrays)
    plan.solve(opt)
    Pg, Xg, sg = plan.read()
    w2 = dict(w, obs_point=w["obs_point"][of > -10], obs_frame=of[of > -10], obs_uv=w["obs_uv"][of > -10])
    Ph, Xh, sh = ctx.ba_local([w2], opt)
    assert close(Pg[0], Ph[0]) and close(Xg[0], Xh[0])
    dp = ctx.empty((10, 6), np.float32)
    plan.result_dev(dp, None)
    assert np.array_equal(dp.numpy(), Pg[0].astype(np.float32))
    plan.close()
    dp.free()
    for a in arrays.values():
        a.free()
