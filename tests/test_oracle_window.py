"""CPU: oracle windowed matchers pinned against the independent pure-Python restatement."""
import numpy as np
import pytest

import oracle as O
import pyref
from lorb_slam_amd import synth


@pytest.mark.parametrize("seed", [5, 6])
def test_local_points_oracle_vs_pyref(seed):
    pr = synth.local_points_problem(seed=seed, n_kps=400, n_pts=500, n_true=250)
    a, n = O.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 1.0)
    b, m = pyref.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 1.0)
    assert n == m
    assert np.array_equal(np.where(a >= 0, a, -1), b)


def test_features_in_area_vs_pyref():
    pr = synth.local_points_problem(seed=3, n_kps=600, n_pts=10, n_true=5)
    fp, kps = pr["fp"], pr["kps"]
    grid = pyref.build_grid(fp, kps)
    rng = np.random.default_rng(0)
    for _ in range(200):
        x, y = rng.uniform(-20, 780), rng.uniform(-20, 500)
        r = float(np.float32(rng.uniform(1, 30)))
        lo, hi = int(rng.integers(-1, 4)), int(rng.integers(-1, 8))
        got = O.features_in_area(fp, kps, np.float32(x), np.float32(y), np.float32(r), lo, hi)
        ref = pyref.features_in_area(fp, kps, grid, x, y, r, lo, hi)
        assert list(got) == ref


def test_frame_match_oracle_runs():
    s = synth.two_frames(seed=1)
    a, n = O.search_by_projection_frame(s["fp"], s["cur_Tcw"], s["cur_kps"], s["slot_state"], s["last"], 15.0)
    assert n > 100  # most of the 200 shared points are recovered at th=15
    assert (a >= -2).all()


def test_inv4_and_unproject():
    T = synth.Tcw_from([0.1, -0.2, 0.05], [0.3, -0.1, 0.5])
    Ti, ok = O.inv4_f32(T)
    assert ok and np.allclose(Ti @ T, np.eye(4), atol=1e-6)
    fp = synth.frame_params()
    out = O.unproject_stereo(fp, T, [100.0, 300.0], [50.0, 200.0], [2.0, -1.0])
    assert np.array_equal(out[1], np.zeros(3, np.float32))
    Xc = T.astype(np.float64) @ np.array([*out[0], 1.0])   # back into the camera frame
    assert abs(Xc[2] - 2.0) < 1e-5
    assert abs(Xc[0] - (100.0 - fp["cx"]) * 2.0 / fp["fx"]) < 1e-4


def test_track_local_map_oracle_chain():
    """The EstimatePoseLocal chain (frustum → skip mask → local search) on the synthetic local map is
    non-trivial: many points in view, skipped points masked, many matches."""
    pr = synth.local_map_problem(seed=11)
    fr, assign, nm = O.track_local_map(pr["fp"], pr["Tcw"], pr["kps"], pr["slot_state"], pr["pts"], 0.5, 1.0)
    skip = pr["pts"]["in_frame"].astype(bool) | pr["pts"]["is_bad"].astype(bool)
    assert fr["in_view"][skip].sum() == 0
    assert fr["in_view"].sum() > 1000
    assert nm > 300
    assert (assign >= 0).sum() == nm


@pytest.mark.parametrize("seed", [21, 22])
def test_stereo_oracle_vs_pyref(seed):
    """ComputeStereoMatches: C restatement == independent pure-Python restatement, bit for bit."""
    pr = synth.stereo_problem(seed=seed, n_left=300, n_distract=150, border=4 if seed == 22 else 24)
    a = O.compute_stereo_matches(pr["fp"], pr["left"], pr["right"], pr["pyr_l"], pr["pyr_r"])
    b = pyref.compute_stereo_matches(pr["fp"], pr["left"], pr["right"], pr["pyr_l"], pr["pyr_r"])
    assert a[2] == b[2] and a[2] > 100
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_orb_oracle_vs_pyref():
    """ORB descriptor stage: C restatement == independent numpy/scipy restatement (blur via
    scipy.ndimage mirror correlation, moments via numpy), bit for bit."""
    pr = synth.orb_problem(seed=31, n_kps=120)
    for lv in (0, 3, 7):
        assert np.array_equal(O.orb_blur(pr["pyr"][lv]), pyref.orb_blur(pr["pyr"][lv]))
    a = O.orb_describe(pr["pyr"], pr["x"], pr["y"], pr["level"], pr["pattern"])
    b = pyref.orb_describe(pr["pyr"], pr["x"], pr["y"], pr["level"], pr["pattern"])
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[1], b[1])
    assert O.orb_gauss_kernel().tolist() == [18, 34, 49, 55, 49, 34, 18]
    assert O.orb_umax().tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    for yx in [(1.0, 1.0), (-3.0, 2.0), (0.0, -5.0), (7.5, -0.25), (0.0, 0.0)]:
        assert O.fast_atan2(*yx) == pyref.fast_atan2(*yx)


@pytest.mark.parametrize("th", [7, 20])
def test_fast_oracle_vs_pyref(th):
    """cv::FAST restatement (C) == independent numpy restatement on textured images."""
    pr = synth.orb_problem(seed=41, n_kps=1)
    for lv in (0, 4):
        img = pr["pyr"][lv][:90, :130]
        a = O.fast(img, th)
        b = pyref.fast(img, th)
        assert len(a[0]) > 10
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


def test_orb_cells_layout():
    """ComputeKeyPointsOctTree's grid (src/ORBextractor.cpp:803-847): C restatement == Python one;
    752 x 480 level 0 has 24 x 14 cells of 30 x 32 pixels (+6 overlap)."""
    nd = O.orb_features_per_level(1000)
    assert nd.sum() == 1000 and nd[0] == 217
    for shape in ((480, 752), (400, 667), (134, 210), (97, 131)):
        c, nc, nr = O.orb_cells(*shape)
        assert [tuple(x) for x in c] == pyref.orb_cells(*shape), shape
    c, nc, nr = O.orb_cells(480, 752)
    assert (nc, nr) == (24, 14) and tuple(c[0]) == (16, 16, 36, 38)
    pr = synth.orb_problem(seed=42, n_kps=1)
    out = O.orb_fast_cells(pr["pyr"])
    assert len(out["x"]) > 1000 and out["cell_base"][-1] > 8


@pytest.mark.parametrize("seed,kind", [(43, "noise"), (91, "scene"), (92, "scene")])
def test_distribute_octree_oracle_vs_pyref(seed, kind):
    """DistributeOctTree (src/ORBextractor.cpp:554-797): the C restatement (linked list) equals the
    Python one (list insert(0, ...)) on every level, at several N (incl. N above the key count and
    the focused loop's break)."""
    pyr = (synth.orb_problem(seed=seed, n_kps=1)["pyr"] if kind == "noise"
           else O.orb_pyramid(synth.orb_scene(seed=seed), synth.scale_factors()))
    f = O.orb_fast_cells(pyr)
    for l, p in enumerate(pyr):
        b0, b1 = f["cell_off"][f["cell_base"][l] + l], f["cell_off"][f["cell_base"][l + 1] + l]
        kx, ky, kr = f["x"][b0:b1] - 16, f["y"][b0:b1] - 16, f["response"][b0:b1]
        for N in (1, 37, 217, 5000):
            a = O.distribute_octree(kx, ky, kr, 16, p.shape[1] - 16, 16, p.shape[0] - 16, N)
            b = pyref.distribute_octree(kx, ky, kr, 16, p.shape[1] - 16, 16, p.shape[0] - 16, N)
            assert np.array_equal(a, b), (l, N)
            assert len(a) >= min(N, 1) and len(set(a.tolist())) == len(a)


def test_distribute_octree_edges():
    """Empty input, one key, duplicate keys at one position (overlapping cells) and keys on the
    split lines."""
    e = np.zeros(0, np.float32)
    assert len(O.distribute_octree(e, e, e, 16, 736, 16, 464, 100)) == 0
    one = np.array([5.0], np.float32)
    assert O.distribute_octree(one, one, one, 16, 736, 16, 464, 100).tolist() == [0]
    x = np.array([100, 100, 100, 360, 360, 360, 359, 0], np.float32)
    y = np.array([50, 50, 50, 224, 224, 223, 224, 0], np.float32)
    r = np.array([3, 9, 9, 1, 2, 2, 5, 4], np.float32)
    for N in (1, 2, 4, 8, 100):
        a = O.distribute_octree(x, y, r, 16, 736, 16, 464, N)
        assert np.array_equal(a, pyref.distribute_octree(x, y, r, 16, 736, 16, 464, N)), N


def test_orb_detect_oracle():
    """ComputeKeyPointsOctTree: per level about n_desired keypoints (the quadtree may overshoot by
    up to 3), all at the level's octave and inside its 16-pixel border."""
    pr = synth.orb_problem(seed=43, n_kps=1)
    nd = O.orb_features_per_level(1000)
    d = O.orb_detect(pr["pyr"], nd, synth.scale_factors())
    lo = d["level_off"]
    for l in range(8):
        assert nd[l] <= lo[l + 1] - lo[l] <= nd[l] + 3
        assert (d["octave"][lo[l]:lo[l + 1]] == l).all()
        h, w = pr["pyr"][l].shape
        assert (d["x"][lo[l]:lo[l + 1]] >= 19).all() and (d["x"][lo[l]:lo[l + 1]] <= w - 20).all()
    assert lo[-1] >= 1000


def test_resize_oracle_vs_pyref():
    """OpenCV 3.1 8U linear resize: C restatement == numpy restatement; a constant stays constant;
    a horizontal ramp resamples within 1 grey level of the exact linear interpolation."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(97, 131), dtype=np.uint8)
    for h, w in ((81, 109), (67, 91), (40, 56)):
        assert np.array_equal(O.resize_linear(img, h, w), pyref.resize_linear(img, h, w))
    assert (O.resize_linear(np.full((50, 70), 77, np.uint8), 42, 58) == 77).all()
    ramp = np.tile(np.arange(200, dtype=np.float64), (20, 1)).astype(np.uint8)
    out = O.resize_linear(ramp, 17, 167).astype(np.float64)
    xs = (np.arange(167) + 0.5) * (200 / 167) - 0.5
    assert np.abs(out[5] - np.clip(xs, 0, 199)).max() <= 1.0
    pyr = O.orb_pyramid(img, synth.scale_factors())
    assert [p.shape for p in pyr[:3]] == [(97, 131), (81, 109), (67, 91)]
