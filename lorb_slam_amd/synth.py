"""Seeded synthetic workloads for the LORB_SLAM hot path.

No dataset ships with the reference and there is no network, so every benchmark
and parity test runs on these generators.  Geometry follows the EuRoC-like intrinsics the
reference reads from EuRoC.yaml (src/camera.cpp:38-42); ORB level statistics follow
ORBextractor's per-level feature split (src/ORBextractor.cpp:412-485).
"""
import math

import numpy as np

W, H = 752, 480
FX = FY = 435.2
CX, CY = 367.5, 252.2
BF = 47.9
N_LEVELS = 8
SCALE = 1.2


def scale_factors(n_levels=N_LEVELS, scale=SCALE):
    sf = [np.float32(1.0)]
    for _ in range(1, n_levels):
        sf.append(np.float32(sf[-1] * np.float32(scale)))  # ORBextractor: float recurrence
    return np.array(sf, np.float32)


def frame_params(fx=FX, fy=FY, cx=CX, cy=CY, bf=BF, width=W, height=H):
    """Frame fields as ComputeImageBounds / the Frame ctor set them (src/frame.cpp:31-36, 67-85)."""
    f32 = np.float32
    min_x, max_x, min_y, max_y = f32(0), f32(width), f32(0), f32(height)
    return dict(fx=f32(fx), fy=f32(fy), cx=f32(cx), cy=f32(cy), bf=f32(bf), b=f32(f32(bf) / f32(fx)),
                min_x=min_x, max_x=max_x, min_y=min_y, max_y=max_y,
                grid_w_inv=f32(f32(64) / (max_x - min_x)), grid_h_inv=f32(f32(48) / (max_y - min_y)),
                n_levels=N_LEVELS, log_scale_factor=np.float32(math.log(np.float32(SCALE))),
                scale_factors=scale_factors())


def level_probs(n_levels=N_LEVELS, scale=SCALE):
    f = 1.0 / scale
    w = np.array([f ** l for l in range(n_levels)])
    return w / w.sum()


def random_desc(rng, n):
    return rng.integers(0, 256, size=(n, 32), dtype=np.uint8)


def flip_bits(rng, desc, max_flips):
    """copy of desc with U{0..max_flips} random distinct bit flips per row"""
    out = desc.copy()
    n = len(desc)
    nf = rng.integers(0, max_flips + 1, size=n)
    for i in range(n):
        if nf[i]:
            bits = rng.choice(256, size=nf[i], replace=False)
            for b in bits:
                out[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return out


def bf_problem(seed=2, nq=2000, nt=2000, n_planted=1000, max_flips=32, random_levels=False):
    """BASELINE config 1: Nq=Nt=2000 random 256-bit descriptors, n_planted trains are bit-flipped
    copies of random queries."""
    rng = np.random.default_rng(seed)
    q = random_desc(rng, nq)
    t = random_desc(rng, nt)
    src = rng.choice(nq, size=min(n_planted, nt), replace=False)
    dst = rng.choice(nt, size=len(src), replace=False)
    t[dst] = flip_bits(rng, q[src], max_flips)
    lev = rng.choice(N_LEVELS, size=nt, p=level_probs()).astype(np.int32) if random_levels else np.zeros(nt, np.int32)
    return q, t, lev


def rodrigues(aa):
    aa = np.asarray(aa, np.float64)
    th = np.linalg.norm(aa)
    if th < 1e-300:
        return np.eye(3)
    k = aa / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def Tcw_from(aa, t):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = rodrigues(aa)
    T[:3, 3] = t
    return T


# ------------------------------------------------------------------------------------------
def ba_window(seed=3, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400, obs_lens=(7, 8),
              noise_px=0.5, fx=FX, fy=FY, cx=CX, cy=CY, pert=(2e-3, 2e-2, 5e-2), point_order="first_kf"):
    """Local-BA window.  KF i: camera centre (0.1 i, 0, 0), yaw 0.01 i.
    Each point is seen by a contiguous KF range of length obs_lens[p % len]; n_fixed extra
    out-of-window KFs (MPCost, fixed pose) each observe ~fixed_obs_per_kf points to fix the gauge.
    point_order "first_kf" numbers the points by their first observing window keyframe, oldest
    first (stable).  That is a synthetic order with camera locality, NOT the reference's order:
    BA::LocalPoseOptimization collects points frame by frame starting from the CURRENT frame, then
    its covisible frames in GetCovisibleFrames() order (src/bundle_adjust.cpp:208-241,
    src/frame.cpp:729), each frame's map points not seen before.  The device-built plans of the
    chained map step take the reference's order (tests/test_gpu_ba.py reference_camera_order);
    "random" keeps the draw order (no camera locality; test_local_ba_point_order_without_camera_
    locality).  Bench windows before round 5 used "random".
    Returns the problem dict consumed by lorb_ba_local / or_ba_local plus ground truth."""
    rng = np.random.default_rng(seed)

    def pose_of(i):
        aa = np.array([0.0, 0.01 * i, 0.0])
        R = rodrigues(aa)
        C = np.array([0.1 * i, 0.0, 0.0])
        return aa, -R @ C

    true_poses = np.array([np.concatenate(pose_of(i)) for i in range(n_kf)])
    fixed = np.array([np.concatenate(pose_of(-1 - j)) for j in range(n_fixed)]).reshape(-1, 6)
    pts = np.stack([rng.uniform(-6, 8, n_pts), rng.uniform(-3, 3, n_pts), rng.uniform(4, 20, n_pts)], 1)
    obs_p, obs_f = [], []
    for p in range(n_pts):
        k = obs_lens[p % len(obs_lens)]
        k = min(k, n_kf)
        s = rng.integers(0, n_kf - k + 1)
        for f in range(s, s + k):
            obs_p.append(p); obs_f.append(f)
    for j in range(n_fixed):
        sel = rng.choice(n_pts, size=min(fixed_obs_per_kf, n_pts), replace=False)
        for p in np.sort(sel):
            obs_p.append(p); obs_f.append(-1 - j)
    obs_p = np.array(obs_p, np.int32); obs_f = np.array(obs_f, np.int32)
    if point_order == "first_kf":  # relabel: point rank by (first window keyframe, draw index)
        first = np.full(n_pts, n_kf, np.int64)
        win = obs_f >= 0
        np.minimum.at(first, obs_p[win], obs_f[win])
        rank = np.empty(n_pts, np.int64)
        rank[np.argsort(first, kind="stable")] = np.arange(n_pts)
        pts = pts[np.argsort(rank)]
        obs_p = rank[obs_p].astype(np.int32)
    elif point_order != "random":
        raise ValueError(point_order)
    allposes = np.concatenate([true_poses, fixed], 0)
    fidx = np.where(obs_f >= 0, obs_f, n_kf + (-1 - obs_f))
    uv = np.zeros((len(obs_p), 2))
    Rs = [rodrigues(allposes[i, :3]) for i in range(len(allposes))]
    for k in range(len(obs_p)):
        pp = Rs[fidx[k]] @ pts[obs_p[k]] + allposes[fidx[k], 3:]
        uv[k] = (fx * pp[0] / pp[2] + cx, fy * pp[1] / pp[2] + cy)
    uv += rng.normal(0, noise_px, uv.shape)
    pose_init = true_poses.copy()
    pose_init[:, :3] += rng.normal(0, pert[0], (n_kf, 3))
    pose_init[:, 3:] += rng.normal(0, pert[1], (n_kf, 3))
    point_init = pts + rng.normal(0, pert[2], pts.shape)
    return dict(pose_init=pose_init.astype(np.float32), fixed_pose=fixed.astype(np.float32),
                point_init=point_init.astype(np.float32), obs_point=obs_p, obs_frame=obs_f,
                obs_uv=uv.astype(np.float32), intr=(np.float32(fx), np.float32(fy), np.float32(cx), np.float32(cy)),
                true_poses=true_poses, true_points=pts)


def reference_window_order(win, curr=None):
    """The window as BA::LocalPoseOptimization assembles it (src/bundle_adjust.cpp:210-220): the
    current keyframe first, then GetCovisibleFrames() -- the connected keyframes sorted by ASCENDING
    covisibility weight (shared map points; src/frame.cpp:754-774, 851), ties by keyframe index.
    Returns (window with its poses / observation frames relabelled, order) where order[i] is the
    original pose index of window pose i."""
    n = len(win["pose_init"])
    curr = n - 1 if curr is None else curr
    opt = win["obs_frame"] >= 0
    pts_of = [set(win["obs_point"][opt & (win["obs_frame"] == f)].tolist()) for f in range(n)]
    weight = [len(pts_of[curr] & pts_of[f]) for f in range(n)]
    others = sorted((f for f in range(n) if f != curr), key=lambda f: (weight[f], f))
    order = np.array([curr] + others, np.int64)
    pos = np.empty(n, np.int64)
    pos[order] = np.arange(n)
    out = dict(win)
    out["pose_init"] = win["pose_init"][order].copy()
    out["obs_frame"] = np.where(opt, pos[np.maximum(win["obs_frame"], 0)], win["obs_frame"]).astype(np.int32)
    if "true_poses" in win:
        out["true_poses"] = win["true_poses"][order].copy()
    return out, order


def pose_only_batch(seed=1, n_frames=1, n_res=200, fx=FX, fy=FY, cx=CX, cy=CY, quirk=True, noise_px=0.5):
    """BA::ProjectPoseOptimization problems: n_res matched map points per frame,
    observation = reprojection + N(0, noise_px).  quirk=True passes fy_eff = fx (PoseCost uses fx
    for v, src/bundle_adjust.cpp:51) to the solver, as the reference does."""
    rng = np.random.default_rng(seed)
    res_off = [0]
    intr, pose_init, pts3d, obs2d = [], [], [], []
    for f in range(n_frames):
        aa = np.array([0.01, -0.005, 0.002]) + rng.normal(0, 0.01, 3)
        t = np.array([0.05, 0.0, 0.02]) + rng.normal(0, 0.05, 3)
        R = rodrigues(aa)
        X = np.stack([rng.uniform(-4, 4, n_res), rng.uniform(-2.5, 2.5, n_res), rng.uniform(2, 10, n_res)], 1)
        Xc = X @ R.T + t
        fyv = fx if quirk else fy
        uv = np.stack([fx * Xc[:, 0] / Xc[:, 2] + cx, fyv * Xc[:, 1] / Xc[:, 2] + cy], 1)
        uv += rng.normal(0, noise_px, uv.shape)
        pi = np.concatenate([aa + rng.normal(0, 5e-3, 3), t + rng.normal(0, 3e-2, 3)])
        intr.append([fx, fyv, cx, cy]); pose_init.append(pi); pts3d.append(X); obs2d.append(uv)
        res_off.append(res_off[-1] + n_res)
    return dict(res_off=np.array(res_off, np.int32), intr=np.array(intr, np.float32),
                pose_init=np.array(pose_init, np.float32), pts3d=np.concatenate(pts3d).astype(np.float32),
                obs2d=np.concatenate(obs2d).astype(np.float32))


# ------------------------------------------------------------------------------------------
def _project(T, X, fp):
    Xc = (T[:3, :3].astype(np.float64) @ X.T).T + T[:3, 3]
    u = fp["fx"] * Xc[:, 0] / Xc[:, 2] + fp["cx"]
    v = fp["fy"] * Xc[:, 1] / Xc[:, 2] + fp["cy"]
    return np.stack([u, v], 1), Xc[:, 2]


def two_frames(seed=1, n_kps=500, n_shared=200, locked_frac=0.5, with_stereo=True, prefilled=0):
    """frame A (last) and B (current), n_kps each, n_shared map points of A are
    re-observed in B (reprojection + N(0,0.5px), descriptor with U{0..12} bit flips).
    Returns inputs for Matcher::SearchByProjection(curr, last, th) (a4) and the BF match (a2)."""
    rng = np.random.default_rng(seed)
    fp = frame_params()
    TA = Tcw_from([0, 0, 0], [0, 0, 0])
    TB = Tcw_from([0.01, -0.005, 0.002], [0.05, 0.0, 0.02])
    probs = level_probs()
    # last frame
    descA = random_desc(rng, n_kps)
    octA = rng.choice(N_LEVELS, size=n_kps, p=probs).astype(np.int32)
    angA = rng.uniform(0, 360, n_kps).astype(np.float32)
    has_mp = np.zeros(n_kps, np.uint8)
    mp_idx = rng.choice(n_kps, size=n_shared, replace=False)
    has_mp[mp_idx] = 1
    # extra map points in A that are NOT observed in B (plenty of non-matches)
    extra = rng.choice(np.setdiff1d(np.arange(n_kps), mp_idx), size=min(n_kps - n_shared, n_shared // 2), replace=False)
    has_mp[extra] = 1
    Xw = np.stack([rng.uniform(-5, 5, n_kps), rng.uniform(-3, 3, n_kps), rng.uniform(2, 10, n_kps)], 1).astype(np.float32)
    mp_locked = (rng.uniform(size=n_kps) < locked_frac).astype(np.uint8)
    outlier = (rng.uniform(size=n_kps) < 0.02).astype(np.uint8)
    # current frame
    uvB, zB = _project(TB, Xw[mp_idx].astype(np.float64), fp)
    uvB += rng.normal(0, 0.5, uvB.shape)
    xB = rng.uniform(0, W, n_kps).astype(np.float32)
    yB = rng.uniform(0, H, n_kps).astype(np.float32)
    descB = random_desc(rng, n_kps)
    octB = rng.choice(N_LEVELS, size=n_kps, p=probs).astype(np.int32)
    angB = rng.uniform(0, 360, n_kps).astype(np.float32)
    slots = rng.choice(n_kps, size=n_shared, replace=False)
    xB[slots] = np.clip(uvB[:, 0], 0, W - 1e-3); yB[slots] = np.clip(uvB[:, 1], 0, H - 1e-3)
    descB[slots] = flip_bits(rng, descA[mp_idx], 12)
    octB[slots] = np.clip(octA[mp_idx] + rng.integers(-1, 2, n_shared), 0, N_LEVELS - 1)
    angB[slots] = np.mod(angA[mp_idx] - rng.normal(5.0, 3.0, n_shared), 360).astype(np.float32)
    uR = np.full(n_kps, -1.0, np.float32)
    if with_stereo:
        has_st = rng.uniform(size=n_kps) < 0.6
        depth = rng.uniform(2, 10, n_kps).astype(np.float32)
        depth[slots] = zB.astype(np.float32)
        uR[has_st] = (xB[has_st] - fp["bf"] / depth[has_st]).astype(np.float32)
    slot_state = np.zeros(n_kps, np.uint8)
    if prefilled:
        pf = rng.choice(n_kps, size=prefilled, replace=False)
        slot_state[pf] = rng.integers(1, 3, size=prefilled).astype(np.uint8)
    cur_kps = dict(x=xB, y=yB, octave=octB, angle=angB, u_right=uR, desc=descB)
    last = dict(Tcw=TA, has_mp=has_mp, outlier=outlier, mp_locked=mp_locked, mp_pos=Xw,
                mp_desc=descA, octave=octA, angle=angA)
    return dict(fp=fp, cur_Tcw=TB, cur_kps=cur_kps, slot_state=slot_state, last=last)


def local_points_problem(seed=5, n_kps=2000, n_pts=3000, n_true=1500, locked_frac=0.8, slot_prefill=100):
    """Inputs of Matcher::SearchByProjection(F, set<MapPoint*>, th) (a5): a frame with n_kps
    keypoints and n_pts local map points already projected by IsInFrustum (the tracking
    fields), n_true of them re-observing a keypoint (bit-flipped descriptor)."""
    rng = np.random.default_rng(seed)
    fp = frame_params()
    probs = level_probs()
    x = rng.uniform(0, W, n_kps).astype(np.float32)
    y = rng.uniform(0, H, n_kps).astype(np.float32)
    octv = rng.choice(N_LEVELS, size=n_kps, p=probs).astype(np.int32)
    ang = rng.uniform(0, 360, n_kps).astype(np.float32)
    desc = random_desc(rng, n_kps)
    uR = np.full(n_kps, -1.0, np.float32)
    st = rng.uniform(size=n_kps) < 0.5
    uR[st] = (x[st] - rng.uniform(3, 20, st.sum())).astype(np.float32)
    pdesc = random_desc(rng, n_pts)
    px = rng.uniform(0, W, n_pts).astype(np.float32)
    py = rng.uniform(0, H, n_pts).astype(np.float32)
    plev = rng.choice(N_LEVELS, size=n_pts, p=probs).astype(np.int32)
    tk = rng.choice(n_kps, size=n_true, replace=False)
    tp = rng.choice(n_pts, size=n_true, replace=False)
    px[tp] = x[tk] + rng.normal(0, 1.0, n_true).astype(np.float32)
    py[tp] = y[tk] + rng.normal(0, 1.0, n_true).astype(np.float32)
    plev[tp] = np.clip(octv[tk] + rng.integers(0, 2, n_true), 0, N_LEVELS - 1)
    pdesc[tp] = flip_bits(rng, desc[tk], 20)
    pxr = (px - rng.uniform(3, 20, n_pts)).astype(np.float32)
    pxr[tp] = np.where(uR[tk] > 0, uR[tk] + rng.normal(0, 1.0, n_true), pxr[tp]).astype(np.float32)
    vc = rng.uniform(0.5, 1.0, n_pts).astype(np.float32)
    vc[rng.uniform(size=n_pts) < 0.3] = np.float32(0.9995)
    pts = dict(track_in_view=(rng.uniform(size=n_pts) < 0.95).astype(np.uint8),
               is_bad=(rng.uniform(size=n_pts) < 0.01).astype(np.uint8),
               locked=(rng.uniform(size=n_pts) < locked_frac).astype(np.uint8),
               proj_x=px, proj_y=py, proj_xr=pxr, pred_level=plev, view_cos=vc, desc=pdesc)
    slot_state = np.zeros(n_kps, np.uint8)
    if slot_prefill:
        pf = rng.choice(n_kps, size=slot_prefill, replace=False)
        slot_state[pf] = rng.integers(1, 3, size=slot_prefill).astype(np.uint8)
    kps = dict(x=x, y=y, octave=octv, angle=ang, u_right=uR, desc=desc)
    return dict(fp=fp, kps=kps, slot_state=slot_state, pts=pts)


def local_mapping_step(seed=4, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400, n_kps=2000,
                       n_reobs=1500, max_flips=20):
    """BASELINE config "full local_mapping step -- match + triangulate + BA on a 50-KF / 10k-point
    window" (SURVEY §8d C4): the window (ba_window), the window map points' descriptors, and a
    new keyframe with n_kps keypoints of which n_reobs re-observe window map points (bit-flipped
    descriptors) and the rest are new with stereo depth (to be unprojected)."""
    win = ba_window(seed=seed, n_kf=n_kf, n_pts=n_pts, n_fixed=n_fixed, fixed_obs_per_kf=fixed_obs_per_kf)
    rng = np.random.default_rng(seed + 7777)
    mp_desc = random_desc(rng, n_pts)
    kf_desc = random_desc(rng, n_kps)
    re = rng.choice(n_pts, size=n_reobs, replace=False)
    slots = rng.choice(n_kps, size=n_reobs, replace=False)
    kf_desc[slots] = flip_bits(rng, mp_desc[re], max_flips)
    x = rng.uniform(0, W, n_kps).astype(np.float32)
    y = rng.uniform(0, H, n_kps).astype(np.float32)
    depth = np.full(n_kps, -1.0, np.float32)
    new = np.setdiff1d(np.arange(n_kps), slots)
    depth[new] = rng.uniform(2, 20, len(new)).astype(np.float32)
    last = win["true_poses"][-1]
    Tcw = Tcw_from(last[:3], last[3:])
    return dict(window=win, mp_desc=mp_desc, kf_desc=kf_desc, kf_x=x, kf_y=y, kf_depth=depth, kf_Tcw=Tcw,
                reobs_slot=slots, reobs_point=re)


def local_map_problem(seed=7, n_kps=2000, n_pts=3000, n_true=1200, n_in_frame=150, bad_frac=0.01):
    """VisualOdometry::EstimatePoseLocal inputs: a frame with n_kps keypoints
    and n_pts local map points (position, mean viewing normal, scale-invariance distances,
    descriptor, mnObs>0 flag, bad flag, already-matched-in-frame flag); n_true points re-observe a
    keypoint at their projection (bit-flipped descriptor, octave at the predicted level)."""
    rng = np.random.default_rng(seed)
    fp = frame_params()
    T = Tcw_from([0.01, -0.02, 0.005], [0.1, -0.05, 0.2])
    R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
    Ow = -R.T @ t
    x = rng.uniform(0, W, n_kps).astype(np.float32)
    y = rng.uniform(0, H, n_kps).astype(np.float32)
    octv = rng.choice(N_LEVELS, size=n_kps, p=level_probs()).astype(np.int32)
    ang = rng.uniform(0, 360, n_kps).astype(np.float32)
    desc = random_desc(rng, n_kps)
    uR = np.full(n_kps, -1.0, np.float32)
    # map points: mostly in front of the camera, some behind / outside the image
    Xc = np.stack([rng.uniform(-6, 6, n_pts), rng.uniform(-4, 4, n_pts), rng.uniform(-1, 15, n_pts)], 1)
    pos = ((Xc - t) @ R).astype(np.float32)  # world = R^T (Xc - t)
    dist = np.linalg.norm(pos.astype(np.float64) - Ow, axis=1)
    nrm = (pos - Ow) / np.maximum(dist[:, None], 1e-9)
    nrm = (nrm + rng.normal(0, 0.3, nrm.shape) * (rng.uniform(size=(n_pts, 1)) < 0.2)).astype(np.float32)
    maxd = (dist * rng.uniform(1.0, 3.0, n_pts)).astype(np.float32)
    mind = (maxd / np.float32(SCALE ** (N_LEVELS - 1))).astype(np.float32)
    pdesc = random_desc(rng, n_pts)
    # planted re-observations of in-view points
    front = np.where(Xc[:, 2] > 0.5)[0]
    uv = np.stack([FX * Xc[:, 0] / Xc[:, 2] + CX, FY * Xc[:, 1] / Xc[:, 2] + CY], 1)
    inimg = front[(uv[front, 0] > 1) & (uv[front, 0] < W - 1) & (uv[front, 1] > 1) & (uv[front, 1] < H - 1)]
    tp = rng.choice(inimg, size=min(n_true, len(inimg)), replace=False)
    tk = rng.choice(n_kps, size=len(tp), replace=False)
    x[tk] = (uv[tp, 0] + rng.normal(0, 0.7, len(tp))).astype(np.float32)
    y[tk] = (uv[tp, 1] + rng.normal(0, 0.7, len(tp))).astype(np.float32)
    lev = np.clip(np.ceil(np.log(maxd[tp] / dist[tp]) / math.log(SCALE)), 0, N_LEVELS - 1).astype(np.int32)
    octv[tk] = np.clip(lev - rng.integers(0, 2, len(tp)), 0, N_LEVELS - 1)
    desc[tk] = flip_bits(rng, pdesc[tp], 20)
    st = rng.uniform(size=n_kps) < 0.5
    uR[st] = (x[st] - rng.uniform(3, 20, st.sum())).astype(np.float32)
    in_frame = np.zeros(n_pts, np.uint8)
    in_frame[rng.choice(n_pts, size=n_in_frame, replace=False)] = 1
    slot_state = np.zeros(n_kps, np.uint8)
    pf = rng.choice(n_kps, size=100, replace=False)
    slot_state[pf] = rng.integers(1, 3, size=100).astype(np.uint8)
    pts = dict(pos=pos, normal=nrm, max_dist=maxd, min_dist=mind, desc=pdesc,
               locked=(rng.uniform(size=n_pts) < 0.8).astype(np.uint8),
               is_bad=(rng.uniform(size=n_pts) < bad_frac).astype(np.uint8), in_frame=in_frame)
    kps = dict(x=x, y=y, octave=octv, angle=ang, u_right=uR, desc=desc)
    return dict(fp=fp, Tcw=T, kps=kps, slot_state=slot_state, pts=pts)


def _bilinear(img, x, y):
    h, w = img.shape
    x = np.clip(x, 0, w - 1.001); y = np.clip(y, 0, h - 1.001)
    x0 = np.floor(x).astype(np.int64); y0 = np.floor(y).astype(np.int64)
    fx, fy = x - x0, y - y0
    a = img[y0, x0] * (1 - fx) + img[y0, x0 + 1] * fx
    b = img[y0 + 1, x0] * (1 - fx) + img[y0 + 1, x0 + 1] * fx
    return a * (1 - fy) + b * fy


def stereo_problem(seed=21, n_left=2000, n_distract=800, frac_true=0.75, width=W, height=H, border=24):
    """Frame::ComputeStereoMatches inputs: a textured scene seen by a rectified pair
    with a smooth disparity field D(x, y) (level-0 pixels), both image pyramids (level l samples the
    scene at scale_factors[l]; right(x, y) = left(x + D, y)), left keypoints with descriptors and
    right keypoints at (x - D, y) + noise with bit-flipped descriptors, plus distractors."""
    rng = np.random.default_rng(seed)
    sf = scale_factors()
    noise = rng.normal(0, 1, (height + 8, width + 80))
    k = np.exp(-0.5 * (np.arange(-4, 5) / 1.4) ** 2); k /= k.sum()
    tex = np.apply_along_axis(lambda r: np.convolve(r, k, "same"), 1, noise)
    tex = np.apply_along_axis(lambda c: np.convolve(c, k, "same"), 0, tex)
    tex = (tex - tex.min()) / (tex.max() - tex.min()) * 255.0

    def disp(x, y):
        return 25.0 + 12.0 * np.sin(x / 90.0) + 8.0 * np.cos(y / 70.0)

    pyr_l, pyr_r = [], []
    for l in range(N_LEVELS):
        s = float(sf[l])
        h, w = int(round(height / s)), int(round(width / s))
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
        X, Y = xx * s + 40.0, yy * s + 4.0
        pyr_l.append(np.clip(np.round(_bilinear(tex, X, Y)), 0, 255).astype(np.uint8))
        pyr_r.append(np.clip(np.round(_bilinear(tex, X + disp(xx * s, yy * s), Y)), 0, 255).astype(np.uint8))
    octv = rng.choice(N_LEVELS, size=n_left, p=level_probs()).astype(np.int32)
    bx = border * sf[octv]
    x = rng.uniform(bx + 40, width - bx).astype(np.float32)
    y = rng.uniform(bx, height - bx).astype(np.float32)
    desc = random_desc(rng, n_left)
    nt = int(n_left * frac_true)
    d = disp(x[:nt].astype(np.float64), y[:nt].astype(np.float64))
    rx = (x[:nt] - d + rng.normal(0, 0.4, nt)).astype(np.float32)
    ry = (y[:nt] + rng.normal(0, 0.6, nt)).astype(np.float32)
    ro = np.clip(octv[:nt] + rng.choice([-1, 0, 0, 0, 1], nt), 0, N_LEVELS - 1).astype(np.int32)
    rdesc = flip_bits(rng, desc[:nt], 30)
    dox = rng.choice(N_LEVELS, size=n_distract, p=level_probs()).astype(np.int32)
    dbx = border * sf[dox]
    right = dict(x=np.concatenate([rx, rng.uniform(dbx, width - dbx).astype(np.float32)]),
                 y=np.concatenate([ry, rng.uniform(dbx, height - dbx).astype(np.float32)]),
                 octave=np.concatenate([ro, dox]), desc=np.concatenate([rdesc, random_desc(rng, n_distract)]))
    perm = rng.permutation(len(right["x"]))
    right = {k_: v[perm] for k_, v in right.items()}
    left = dict(x=x, y=y, octave=octv, desc=desc)
    return dict(fp=frame_params(width=width, height=height), left=left, right=right, pyr_l=pyr_l, pyr_r=pyr_r)


def orb_problem(seed=31, n_kps=2000, width=W, height=H, border=19):
    """ORBextractor descriptor-stage inputs: an 8-level textured pyramid, keypoints
    in level coordinates at least `border` pixels inside their level (EDGE_THRESHOLD = 19), and a
    random 256-pair test pattern with ORB's coordinate range [-13, 12]."""
    rng = np.random.default_rng(seed)
    sp = stereo_problem(seed=seed, n_left=1, n_distract=1, width=width, height=height)
    pyr = sp["pyr_l"]
    lev = rng.choice(N_LEVELS, size=n_kps, p=level_probs()).astype(np.int32)
    rows = np.array([p.shape[0] for p in pyr])[lev]
    cols = np.array([p.shape[1] for p in pyr])[lev]
    x = (border + rng.uniform(0, 1, n_kps) * (cols - 2 * border - 1)).astype(np.float32)
    y = (border + rng.uniform(0, 1, n_kps) * (rows - 2 * border - 1)).astype(np.float32)
    pattern = rng.integers(-13, 13, size=1024).astype(np.int32)
    return dict(pyr=pyr, x=x, y=y, level=lev, pattern=pattern)


def orb_scene(seed=91, rows=H, cols=W, n_shapes=120, noise=3):
    """A camera-like test image for the whole ORB extractor: a smooth background
    gradient, random rectangles and discs of random grey levels (corners and edges of every
    orientation), a few noise-textured patches (dense FAST responses, many equal scores), and
    small pixel noise.  uint8, rows x cols."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:rows, 0:cols].astype(np.float64)
    img = 90 + 40 * np.sin(xx / 97.0) + 30 * np.cos(yy / 71.0)
    for _ in range(n_shapes):
        v = rng.uniform(0, 255)
        if rng.uniform() < 0.6:
            x0, y0 = rng.uniform(-40, cols), rng.uniform(-40, rows)
            w, h = rng.uniform(8, 120), rng.uniform(8, 90)
            m = (xx >= x0) & (xx < x0 + w) & (yy >= y0) & (yy < y0 + h)
        else:
            cx, cy, r = rng.uniform(0, cols), rng.uniform(0, rows), rng.uniform(5, 50)
            m = (xx - cx) ** 2 + (yy - cy) ** 2 < r * r
        img[m] = v
    for _ in range(6):
        x0, y0 = int(rng.uniform(0, cols - 80)), int(rng.uniform(0, rows - 60))
        img[y0:y0 + 60, x0:x0 + 80] += rng.normal(0, 25, (60, 80))
    img += rng.integers(-noise, noise + 1, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def mapping_sequence(seed=4, n_kf=50, n_fixed=5, n_new=189, obs_lens=(7, 8), steps=8, n_kps=2000,
                     max_flips=20, noise_px=0.5, pert=(2e-3, 2e-2, 5e-2), fx=FX, fy=FY, cx=CX, cy=CY):
    """A stationary keyframe stream for the LocalMapping full step (VERDICT r01
    item 3).  Keyframe t: camera centre (0.1 t, 0, 0), yaw 0.01 t.  Keyframe t creates n_new map
    points, each seen by the contiguous keyframe range [t, t + L), L in obs_lens -- so a 50-KF window
    holds ~10k points and ~77k observations at every step.

    Returns dict(init=..., steps=[...]):
      init: the window before the first step -- optimised keyframes [0, n_kf), fixed [-n_fixed, 0):
            pose_init (perturbed) / fixed_pose (float rvec|tvec), points (perturbed positions), their
            descriptors, and every observation (point, keyframe id, uv) of a point seen by an
            optimised keyframe, point-major;
      steps[i]: keyframe n_kf + i: its tracked pose (perturbed truth; rvec|tvec and Tcw as float),
            n_kps keypoints (x, y, 32-byte descriptors, stereo depth) -- re-observations of the
            map's points (descriptor of the point with U{0..max_flips} flipped bits, depth -1), the
            keyframe's new points (depth > 0: to be unprojected) and random distractors (depth -1).
    A point's descriptor is the one of the keypoint that created it (random for initial points)."""
    rng = np.random.default_rng(seed)

    def pose_of(t):
        aa = np.array([0.0, 0.01 * t, 0.0])
        R = rodrigues(aa)
        return aa, -R @ np.array([0.1 * t, 0.0, 0.0])

    lmax = max(obs_lens)
    first = -n_fixed - lmax + 1
    last = n_kf + steps
    # points: creation keyframe, length, true position in front of the creating camera's view
    created, length, X = [], [], []
    for t in range(first, last):
        aa, tt = pose_of(t)
        R = rodrigues(aa)
        C = -R.T @ tt
        for _ in range(n_new):
            L = obs_lens[len(created) % len(obs_lens)]
            # a point visible from keyframes t .. t+L-1: ahead of the cameras, inside the image
            z = rng.uniform(4, 20)
            u = rng.uniform(40, W - 40); v = rng.uniform(40, H - 40)
            pc = np.array([(u - cx) / fx * z, (v - cy) / fy * z, z])
            X.append(R.T @ (pc - tt))
            created.append(t); length.append(L)
    created = np.array(created); length = np.array(length); X = np.array(X)
    n_all = len(X)
    desc = random_desc(rng, n_all)

    def project(t, idx):
        aa, tt = pose_of(t)
        Xc = X[idx] @ rodrigues(aa).T + tt
        return np.stack([fx * Xc[:, 0] / Xc[:, 2] + cx, fy * Xc[:, 1] / Xc[:, 2] + cy], 1), Xc[:, 2]

    def perturbed_pose(t):
        aa, tt = pose_of(t)
        return np.concatenate([aa + rng.normal(0, pert[0], 3), tt + rng.normal(0, pert[1], 3)]).astype(np.float32)

    # initial window: points seen by an optimised keyframe in [0, n_kf)
    vis0 = np.nonzero((created + length > 0) & (created < n_kf))[0]
    obs_p, obs_k, obs_uv = [], [], []
    for t in range(-n_fixed, n_kf):  # keyframe by keyframe, then point-major
        j = np.nonzero((created[vis0] <= t) & (created[vis0] + length[vis0] > t))[0]
        uv, _ = project(t, vis0[j])
        obs_p.append(j); obs_k.append(np.full(len(j), t)); obs_uv.append(uv + rng.normal(0, noise_px, uv.shape))
    obs_p, obs_k, obs_uv = np.concatenate(obs_p), np.concatenate(obs_k), np.concatenate(obs_uv)
    o = np.lexsort((obs_k, obs_p))
    obs_p, obs_k, obs_uv = obs_p[o], obs_k[o], obs_uv[o]
    init = dict(n_kf=n_kf, n_fixed=n_fixed, intr=(np.float32(fx), np.float32(fy), np.float32(cx), np.float32(cy)),
                pose_init=np.array([perturbed_pose(t) for t in range(n_kf)], np.float32),
                fixed_pose=np.array([np.concatenate(pose_of(-1 - j)) for j in range(n_fixed)], np.float32),
                point_init=(X[vis0] + rng.normal(0, pert[2], (len(vis0), 3))).astype(np.float32),
                point_desc=desc[vis0].copy(), point_truth=vis0.copy(),
                obs_point=np.array(obs_p, np.int32), obs_kf=np.array(obs_k, np.int32),
                obs_uv=np.array(obs_uv, np.float32))
    out = []
    for i in range(steps):
        t = n_kf + i
        reob = np.nonzero((created < t) & (created + length > t))[0]
        new = np.nonzero(created == t)[0]
        uv_r, _ = project(t, reob)
        uv_n, z_n = project(t, new)
        n_d = max(0, n_kps - len(reob) - len(new))
        x = np.concatenate([uv_r[:, 0], uv_n[:, 0], rng.uniform(0, W, n_d)]) + np.concatenate(
            [rng.normal(0, noise_px, len(reob) + len(new)), np.zeros(n_d)])
        y = np.concatenate([uv_r[:, 1], uv_n[:, 1], rng.uniform(0, H, n_d)]) + np.concatenate(
            [rng.normal(0, noise_px, len(reob) + len(new)), np.zeros(n_d)])
        kdesc = np.concatenate([flip_bits(rng, desc[reob], max_flips), random_desc(rng, len(new) + n_d)])
        desc[new] = kdesc[len(reob):len(reob) + len(new)]  # a new point takes its keypoint's descriptor
        depth = np.concatenate([np.full(len(reob), -1.0), z_n + rng.normal(0, 0.02, len(new)), np.full(n_d, -1.0)])
        perm = rng.permutation(len(x))  # keypoints in no particular order
        pv = perturbed_pose(t)
        out.append(dict(kf=t, pose=pv, Tcw=Tcw_from(pv[:3].astype(np.float64), pv[3:].astype(np.float64)),
                        x=x[perm].astype(np.float32), y=y[perm].astype(np.float32), desc=kdesc[perm].copy(),
                        depth=depth[perm].astype(np.float32), n_reobs=len(reob), n_new=len(new)))
    return dict(init=init, steps=out)
