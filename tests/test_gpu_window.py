"""GPU parity: windowed matchers (a4/a5), IsInFrustum (a8), UnprojectStereo (a20) vs the oracle.
Match assignments and counts must be bit-exact."""
import os
import numpy as np
import pytest

import oracle as O
import lorb_slam_amd.window  # noqa: F401  (binds Context methods)
from lorb_slam_amd import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,th,prefilled,locked", [(1, 15.0, 0, 0.5), (2, 30.0, 0, 1.0), (3, 15.0, 60, 0.3),
                                                       (4, 5.0, 20, 0.0)])
def test_search_by_projection_frame(ctx, seed, th, prefilled, locked):
    s = synth.two_frames(seed=seed, n_kps=500, n_shared=200, locked_frac=locked, prefilled=prefilled)
    a_g, n_g = ctx.search_by_projection_frame(s["fp"], s["cur_Tcw"], s["cur_kps"], s["slot_state"], s["last"], th)
    a_o, n_o = O.search_by_projection_frame(s["fp"], s["cur_Tcw"], s["cur_kps"], s["slot_state"], s["last"], th)
    assert n_g == n_o
    assert np.array_equal(a_g, a_o)


def test_search_by_projection_frame_large(ctx):
    s = synth.two_frames(seed=9, n_kps=2000, n_shared=1200, locked_frac=0.7, prefilled=100)
    a_g, n_g = ctx.search_by_projection_frame(s["fp"], s["cur_Tcw"], s["cur_kps"], s["slot_state"], s["last"], 15.0)
    a_o, n_o = O.search_by_projection_frame(s["fp"], s["cur_Tcw"], s["cur_kps"], s["slot_state"], s["last"], 15.0)
    assert n_g == n_o and np.array_equal(a_g, a_o)


@pytest.mark.parametrize("seed,n_kps,n_pts,n_true,th", [(5, 2000, 3000, 1500, 1.0), (6, 500, 2000, 400, 1.0),
                                                         (7, 2000, 10000, 1500, 1.0), (8, 1000, 1500, 800, 3.0)])
def test_search_by_projection_local(ctx, seed, n_kps, n_pts, n_true, th):
    pr = synth.local_points_problem(seed=seed, n_kps=n_kps, n_pts=n_pts, n_true=n_true)
    a_g, n_g = ctx.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], th)
    a_o, n_o = O.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], th)
    assert n_g == n_o
    assert np.array_equal(a_g, a_o)


def test_search_by_projection_local_claim_chains(ctx):
    """Many duplicate map points over the same keypoints: long dependency chains through the
    mnObs>0 occupancy rule exercise many fixpoint rounds."""
    pr = synth.local_points_problem(seed=12, n_kps=300, n_pts=200, n_true=150, locked_frac=0.6, slot_prefill=0)
    p = pr["pts"]
    rep = 8
    pts = {k: (np.tile(v, rep) if v.ndim == 1 else np.tile(v, (rep, 1))) for k, v in p.items()}
    rng = np.random.default_rng(0)
    pts["locked"] = (rng.uniform(size=len(pts["locked"])) < 0.6).astype(np.uint8)
    a_g, n_g = ctx.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pts, 1.0)
    a_o, n_o = O.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pts, 1.0)
    assert n_g == n_o and np.array_equal(a_g, a_o)


def _frustum_points(seed, n):
    rng = np.random.default_rng(seed)
    pos = np.stack([rng.uniform(-6, 6, n), rng.uniform(-4, 4, n), rng.uniform(-2, 15, n)], 1).astype(np.float32)
    nrm = rng.normal(size=(n, 3)); nrm[:, 2] = np.abs(nrm[:, 2]) + 1.0
    nrm = (nrm / np.linalg.norm(nrm, axis=1, keepdims=True)).astype(np.float32)
    d = np.linalg.norm(pos, axis=1)
    return dict(pos=pos, normal=nrm, max_dist=(d * rng.uniform(0.8, 3.0, n)).astype(np.float32),
                min_dist=(d * rng.uniform(0.2, 1.0, n) / 3.58).astype(np.float32))


def test_is_in_frustum(ctx):
    fp = synth.frame_params()
    T = synth.Tcw_from([0.02, -0.03, 0.01], [0.1, 0.05, -0.2])
    pts = _frustum_points(3, 20000)
    g = ctx.is_in_frustum(fp, T, pts, 0.5)
    o = O.is_in_frustum(fp, T, pts, 0.5)
    assert np.array_equal(g["in_view"], o["in_view"])
    m = o["in_view"].astype(bool)
    assert m.sum() > 1000
    for k in ("proj_x", "proj_y", "proj_xr", "view_cos"):
        assert np.array_equal(g[k][m], o[k][m]), k
    # predicted level: ceil(logf(ratio)/logScale); GPU logf is (float)log(double) (correctly
    # rounded), glibc logf may differ by 1 ulp -> allow only quotient-at-integer ties
    assert (g["pred_level"][m] != o["pred_level"][m]).sum() == 0


def test_unproject_stereo(ctx):
    fp = synth.frame_params()
    T = synth.Tcw_from([0.02, -0.03, 0.01], [0.1, 0.05, -0.2])
    rng = np.random.default_rng(1)
    n = 5000
    x = rng.uniform(0, 752, n).astype(np.float32); y = rng.uniform(0, 480, n).astype(np.float32)
    d = rng.uniform(-1, 12, n).astype(np.float32)
    assert np.array_equal(ctx.unproject_stereo(fp, T, x, y, d), O.unproject_stereo(fp, T, x, y, d))


@pytest.mark.parametrize("seed,cos_limit,th", [(11, 0.5, 1.0), (12, 0.5, 3.0), (13, 0.8, 1.0)])
def test_track_local_map(ctx, seed, cos_limit, th):
    """lorb_track_local_map_dev vs the oracle chain of EstimatePoseLocal
    (src/visual_odometry.cpp:173-201) -- tracking fields and assignments bit-exact."""
    pr = synth.local_map_problem(seed=seed, bad_frac=0.02)
    g = ctx.track_local_map(pr["fp"], pr["Tcw"], pr["kps"], pr["slot_state"], pr["pts"], cos_limit, th)
    fr, assign, nm = O.track_local_map(pr["fp"], pr["Tcw"], pr["kps"], pr["slot_state"], pr["pts"], cos_limit, th)
    assert np.array_equal(g["in_view"], fr["in_view"])
    m = fr["in_view"].astype(bool)
    assert m.sum() > 500
    for k in ("proj_x", "proj_y", "proj_xr", "view_cos", "pred_level"):
        assert np.array_equal(g[k][m], fr[k][m]), k
    assert g["nmatches"] == nm and nm > 100
    assert np.array_equal(g["assign"], assign)


def test_track_local_map_edges(ctx):
    pr = synth.local_map_problem(seed=14, n_kps=300, n_pts=400, n_true=100)
    fp, T, kps, pts = pr["fp"], pr["Tcw"], pr["kps"], pr["pts"]
    # every point already matched in the frame: nothing in view, no search, nothing assigned
    allin = dict(pts, in_frame=np.ones(400, np.uint8))
    g = ctx.track_local_map(fp, T, kps, None, allin)
    assert g["in_view"].sum() == 0 and g["nmatches"] == 0 and (g["assign"] == -1).all()
    # no map points at all
    empty = {k: v[:0] for k, v in pts.items()}
    g = ctx.track_local_map(fp, T, kps, None, empty)
    assert g["nmatches"] == 0 and (g["assign"] == -1).all()
    # no keypoints: tracking fields still computed
    nok = {k: v[:0] for k, v in kps.items()}
    g = ctx.track_local_map(fp, T, nok, None, pts)
    fr, _, _ = O.track_local_map(fp, T, kps, None, pts)
    assert g["nmatches"] == 0 and np.array_equal(g["in_view"], fr["in_view"])
    # no skip masks (NULL pointers)
    bare = dict(pts, in_frame=None, is_bad=None)
    g = ctx.track_local_map(fp, T, kps, pr["slot_state"], bare)
    fr, assign, nm = O.track_local_map(fp, T, kps, pr["slot_state"], bare)
    assert g["nmatches"] == nm and np.array_equal(g["assign"], assign)


@pytest.mark.parametrize("seed,n_left,n_distract,border,dev", [(21, 2000, 800, 24, False), (22, 2000, 800, 24, True),
                                                               (23, 300, 50, 4, False), (24, 6000, 3000, 10, True)])
def test_compute_stereo_matches(ctx, seed, n_left, n_distract, border, dev):
    """ComputeStereoMatches (src/frame.cpp:125-333) bit-exact vs the oracle, incl.
    keypoints whose SAD windows leave the image (border=4) and the median rejection."""
    pr = synth.stereo_problem(seed=seed, n_left=n_left, n_distract=n_distract, border=border)
    ur, dp = ctx.compute_stereo_matches(pr["fp"], pr["left"], pr["right"], pr["pyr_l"], pr["pyr_r"], device_resident=dev)
    our, odp, npair = O.compute_stereo_matches(pr["fp"], pr["left"], pr["right"], pr["pyr_l"], pr["pyr_r"])
    assert npair > n_left // 3
    assert np.array_equal(ur, our) and np.array_equal(dp, odp)
    assert (ur >= 0).sum() < npair  # the median cut removed some


def test_compute_stereo_matches_edges(ctx):
    pr = synth.stereo_problem(seed=25, n_left=200, n_distract=20)
    fp, L, R, pl, prr = pr["fp"], pr["left"], pr["right"], pr["pyr_l"], pr["pyr_r"]
    # no right keypoints: nothing matched
    noR = {k: v[:0] for k, v in R.items()}
    ur, dp = ctx.compute_stereo_matches(fp, L, noR, pl, prr)
    assert (ur == -1).all() and (dp == -1).all()
    # no left keypoints
    ur, dp = ctx.compute_stereo_matches(fp, {k: v[:0] for k, v in L.items()}, R, pl, prr)
    assert len(ur) == 0
    # a single accepted pair: the median is itself, 2.1 x median keeps it
    one = {k: v[:1] for k, v in L.items()}
    ur, dp = ctx.compute_stereo_matches(fp, one, R, pl, prr)
    o = O.compute_stereo_matches(fp, one, R, pl, prr)
    assert np.array_equal(ur, o[0]) and np.array_equal(dp, o[1])


@pytest.mark.parametrize("seed,n,dev", [(31, 2000, False), (32, 5000, True), (33, 1, False)])
def test_orb_describe(ctx, seed, n, dev):
    """ORB descriptor stage (IC_Angle + GaussianBlur + rBRIEF) bit-exact vs the oracle."""
    pr = synth.orb_problem(seed=seed, n_kps=n)
    ang, desc = ctx.orb_describe(pr["pyr"], pr["x"], pr["y"], pr["level"], pr["pattern"], device_resident=dev)
    oang, odesc = O.orb_describe(pr["pyr"], pr["x"], pr["y"], pr["level"], pr["pattern"])
    assert np.array_equal(ang, oang)
    assert np.array_equal(desc, odesc)


def test_orb_describe_edges(ctx):
    pr = synth.orb_problem(seed=34, n_kps=10)
    ang, desc = ctx.orb_describe(pr["pyr"], pr["x"][:0], pr["y"][:0], pr["level"][:0], pr["pattern"])
    assert len(ang) == 0 and desc.shape == (0, 32)
    x = pr["x"].copy(); x[3] = 5.0  # inside the 19-pixel border: rejected, not read out of bounds
    with pytest.raises(Exception):
        ctx.orb_describe(pr["pyr"], x, pr["y"], pr["level"], pr["pattern"])


@pytest.mark.parametrize("seed,ini,mn", [(51, 20, 7), (52, 40, 7), (53, 60, 7)])
def test_orb_fast_cells(ctx, seed, ini, mn):
    """SURVEY §8f row 3 FAST stage of ComputeKeyPointsOctTree: per-cell FAST + the empty-cell
    minThFAST re-run bit-exact vs the oracle (ini=60 leaves many cells empty at first)."""
    pr = synth.orb_problem(seed=seed, n_kps=1)
    g = ctx.orb_fast_cells(pr["pyr"], ini, mn)
    o = O.orb_fast_cells(pr["pyr"], ini, mn)
    assert np.array_equal(g["cell_base"], o["cell_base"]) and np.array_equal(g["cell_off"], o["cell_off"])
    for k in ("x", "y", "response"):
        assert np.array_equal(g[k], o[k]), k
    assert len(o["x"]) > 1000


@pytest.mark.parametrize("seed,nfeat,kind", [(61, 1000, "noise"), (62, 2000, "noise"), (63, 500, "noise"),
                                             (91, 1000, "scene"), (93, 2000, "scene"), (94, 4000, "scene")])
def test_orb_detect(ctx, seed, nfeat, kind):
    """FAST cells + DistributeOctTree on the device vs the oracle's linked-list
    restatement: keypoints, their order and attributes equal."""
    pyr = (synth.orb_problem(seed=seed, n_kps=1)["pyr"] if kind == "noise"
           else O.orb_pyramid(synth.orb_scene(seed=seed), synth.scale_factors()))
    nd = O.orb_features_per_level(nfeat)
    g = ctx.orb_detect(pyr, nd, synth.scale_factors())
    o = O.orb_detect(pyr, nd, synth.scale_factors())
    for k in ("x", "y", "octave", "size", "response", "level_off"):
        assert np.array_equal(g[k], o[k]), k


@pytest.mark.parametrize("seed,shape", [(71, (480, 752)), (72, (333, 517))])
def test_orb_pyramid(ctx, seed, shape):
    """ComputePyramid (OpenCV 3.1 8U linear resize chain) bit-exact vs the oracle."""
    rng = np.random.default_rng(seed)
    img = synth.orb_problem(seed=seed, n_kps=1)["pyr"][0][:shape[0], :shape[1]]
    img = np.clip(img.astype(np.int32) + rng.integers(-3, 4, img.shape), 0, 255).astype(np.uint8)
    g = ctx.orb_pyramid(img, synth.scale_factors())
    o = O.orb_pyramid(img, synth.scale_factors())
    assert len(g) == len(o) == 8
    for a, b in zip(g, o):
        assert a.shape == b.shape and np.array_equal(a, b)


@pytest.mark.parametrize("nfeat,seed", [(1000, 95), (2000, 96)])
def test_orb_extract_end_to_end(ctx, nfeat, seed):
    """The whole ORBextractor::operator() (src/ORBextractor.cpp:1087-1151) on a 752 x 480 image with
    the reference's bit_pattern_31_: device pipeline (pyramid -> FAST cells -> DistributeOctTree ->
    IC_Angle + blur + rBRIEF -> level-0 coordinates) vs the oracle, bit-exact."""
    import golden_io
    pattern = golden_io.load(os.path.join(os.path.dirname(__file__), "golden", "orb.npz"))["pattern"]
    img = synth.orb_scene(seed=seed)
    sf = synth.scale_factors()
    nd = O.orb_features_per_level(nfeat)
    g = ctx.orb_extract(img, nd, sf, pattern)
    o = O.orb_extract(img, nd, sf, pattern)
    assert len(o["x"]) >= nfeat
    for k in ("x", "y", "octave", "size", "angle", "response", "desc", "level_off"):
        assert np.array_equal(g[k], o[k]), k


def test_orb_and_stereo_argument_errors(ctx):
    """The 8f-row entry points reject malformed inputs with an error instead of reading out of
    bounds: degenerate cell grids, too-small pyramids, pyramids with fewer levels than the frame."""
    from lorb_slam_amd.runtime import LorbError
    pr = synth.orb_problem(seed=81, n_kps=4)
    nd = O.orb_features_per_level(1000)
    with pytest.raises(LorbError):  # a level smaller than one 30-pixel cell inside its border
        ctx.orb_fast_cells([p[:40, :40].copy() for p in pr["pyr"]])
    with pytest.raises(LorbError):  # 1 x 1 levels
        ctx.orb_pyramid(np.zeros((4, 4), np.uint8), synth.scale_factors())
    sp = synth.stereo_problem(seed=82, n_left=50, n_distract=10)
    with pytest.raises(LorbError):  # right pyramid with fewer levels than the frame
        ctx.compute_stereo_matches(sp["fp"], sp["left"], sp["right"], sp["pyr_l"], sp["pyr_r"][:3])
    with pytest.raises(LorbError):  # capacity too small is reported, not overrun
        ctx.orb_detect(pr["pyr"], nd, synth.scale_factors(), max_kp=10)
