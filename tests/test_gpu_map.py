"""GPU parity: the chained LocalMapping step on the HBM-resident map (lorb_map_*, liblorb.so) vs the
oracle's restatement (oracle/oracle_map.py) run on the same slid window.

Per step the oracle starts from the device map's state read back before the step, so each step is
compared from identical inputs: the matcher outputs, the appended / culled / compacted map structure
(point order, descriptors, observations, BA slots) and the observation uv are bit-exact; poses and
points after LocalPoseOptimization's float write-back are within the north_star tolerance 1e-5
relative (|gpu - oracle| <= 1e-5 * max(|oracle|, 1)); the LM summaries agree as in test_gpu_ba."""
import numpy as np
import pytest

from lorb_slam_amd import _abi as A
from lorb_slam_amd import synth
from lorb_slam_amd.runtime import LocalMap, LorbError
from oracle_map import MapOracle
from test_gpu_ba import close, lm_match

pytestmark = pytest.mark.gpu
OPT10 = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                            parameter_tolerance=0.0)
EXACT = ("point_desc", "obs_point", "obs_kf", "obs_uv", "obs_frame")


def same_structure(g, o):
    assert g["t0"] == o["t0"]
    assert g["points"] == o["points"] and g["observations"] == o["observations"], (g["points"], o["points"])
    for k in EXACT:
        assert np.array_equal(g[k], o[k]), k


def run_chain(ctx, seq, opt, n_steps, label="chain", strict=True):
    fp = synth.frame_params()
    M = LocalMap(ctx, seq["init"])
    try:
        g = M.read()
        o = MapOracle(seq["init"]).state()
        same_structure(g, o)
        assert np.array_equal(g["point"], o["point"]) and np.array_equal(g["pose"], o["pose"])
        for i in range(n_steps):
            kf = seq["steps"][i]
            ref = MapOracle.from_state(g, seq["init"]["intr"])
            M.step(fp, kf, opt)
            g = M.read()
            r = ref.step(fp, kf, opt)
            o = ref.state()
            assert np.array_equal(g["match_train"], r["match_train"]), i
            assert g["matches"] == r["n_matches"] and g["new_points"] == r["new_points"]
            assert g["new_observations"] == r["new_observations"]
            same_structure(g, o)
            assert close(g["pose"], o["pose"]), np.abs(g["pose"] - o["pose"]).max()
            assert close(g["point"], o["point"]), np.abs(g["point"] - o["point"]).max()
            assert np.array_equal(g["fixed_pose"], o["fixed_pose"])
            flip = lm_match(g["summary"], r["summary"], gt=M.trace(), ot=r["trace"], label=f"{label} step {i}")
            assert not strict or flip is None, (label, i, flip)
        return M, g
    except BaseException:
        M.close()
        raise


def test_local_mapping_chain_c4(ctx):
    """C4 sizes: 50-KF window + 5 fixed, ~10k points, ~75k observations, 2,000 keypoints per new
    keyframe; 3 consecutive steps"""
    seq = synth.mapping_sequence(steps=3)
    M, g = run_chain(ctx, seq, OPT10, 3)
    info = M.plan_info()
    assert info["cameras"] == 50 and info["band"] <= 47, info
    assert 9000 < g["points"] < 12000 and 60000 < g["observations"] < 90000
    M.close()


def test_local_mapping_chain_c4_ceres_defaults(ctx):
    """the chained C4 step with the options LocalMapping's BA runs with (Ceres
    defaults, src/bundle_adjust.cpp:308-314): 3 steps, each step's termination, accepted steps and
    per-iteration outcomes as the oracle's (strict)."""
    seq = synth.mapping_sequence(steps=3)
    M, g = run_chain(ctx, seq, A.LMOptions.default(), 3, label="map c4 defaults")
    M.close()


def test_local_mapping_chain_default_options(ctx):
    """Ceres default options (tolerances on), a small window"""
    seq = synth.mapping_sequence(seed=9, n_kf=12, n_fixed=3, n_new=60, obs_lens=(4, 5), steps=3, n_kps=600)
    M, _ = run_chain(ctx, seq, A.LMOptions.default(), 3)
    M.close()


def test_local_mapping_ragged_keyframes(ctx):
    """a keyframe without keypoints, one without stereo depth, then a normal one"""
    seq = synth.mapping_sequence(seed=5, n_kf=10, n_fixed=2, n_new=40, obs_lens=(3, 4), steps=3, n_kps=300)
    k0, k1 = seq["steps"][0], seq["steps"][1]
    seq["steps"][0] = dict(k0, x=k0["x"][:0], y=k0["y"][:0], desc=k0["desc"][:0], depth=k0["depth"][:0])
    seq["steps"][1] = dict(k1, depth=np.full_like(k1["depth"], -1.0))
    M, g = run_chain(ctx, seq, OPT10, 3)
    M.close()


def test_local_mapping_capacity_error(ctx):
    """a step that would overflow the map's point capacity is refused and leaves the map unchanged;
    the next step (a keyframe without stereo depth: matches only, no new points) runs from the
    unchanged map and equals the oracle's step from the same state"""
    seq = synth.mapping_sequence(seed=5, n_kf=10, n_fixed=2, n_new=40, obs_lens=(3, 4), steps=2, n_kps=300)
    n_pts = len(seq["init"]["point_init"])
    fp = synth.frame_params()
    M = LocalMap(ctx, seq["init"], max_points=n_pts + 5, max_keypoints=512)
    try:
        before = M.read()
        with pytest.raises(LorbError, match="capacity"):
            M.step(fp, seq["steps"][0], OPT10)
        after = M.read()
        same_structure(after, before)
        for k in ("point", "pose", "fixed_pose"):
            assert np.array_equal(after[k], before[k]), k
        assert after["new_points"] == 0 and after["new_observations"] == 0
        k1 = dict(seq["steps"][1], depth=np.full_like(seq["steps"][1]["depth"], -1.0))
        ref = MapOracle.from_state(after, seq["init"]["intr"])
        M.step(fp, k1, OPT10)
        g = M.read()
        r = ref.step(fp, k1, OPT10)
        o = ref.state()
        assert np.array_equal(g["match_train"], r["match_train"])
        assert g["new_points"] == 0 and g["matches"] == r["n_matches"]
        same_structure(g, o)
        assert close(g["pose"], o["pose"]) and close(g["point"], o["point"])
        lm_match(g["summary"], r["summary"])
    finally:
        M.close()


def test_local_mapping_overlapped_chain_bit_identical(ctx):
    """The bench's timed regime: C4 keyframes issued back to back through
    step_dev with the overlap on (step t+1's crossCheck + append on the map's own stream under step
    t's LM solve and write-back) and no host synchronisation in between, then the map read once.  A
    second map runs the same keyframes serially (overlap off) and is checked against the oracle after
    every step (run_chain).  Done when the overlapped map equals the serial one bit for bit --
    structure, descriptors, poses, points, LM summary -- and every serial step matches the oracle
    (structure bit-exact, poses / points within 1e-5)."""
    n = 6
    seq = synth.mapping_sequence(steps=n)
    fp = A.make_frame_params(synth.frame_params())
    # the keyframe arrays, complete in HBM before the first step (lorb_map_set_overlap's requirement)
    dev = [(k["pose"], k["Tcw"], len(k["x"]), ctx.to_device(A.u8(k["desc"])), ctx.to_device(A.f32(k["x"])),
            ctx.to_device(A.f32(k["y"])), ctx.to_device(A.f32(k["depth"]))) for k in seq["steps"][:n]]
    ctx.sync()
    Mo = LocalMap(ctx, seq["init"])
    Ms = None
    try:
        Mo.set_overlap(True)
        for pose, Tcw, nk, dd, dx, dy, dz in dev:
            Mo.step_dev(fp, pose, Tcw, nk, dd, dx, dy, dz, OPT10)
        go = Mo.read()
        # every step after the first found the previous step's plan built: n - 1 ran overlapped
        assert go["overlapped_steps"] == n - 1, go["overlapped_steps"]
        Ms, gs = run_chain(ctx, seq, OPT10, n)
        assert gs["overlapped_steps"] == 0
        for k in ("t0", "points", "observations", "keypoints", "new_points", "new_observations", "matches"):
            assert go[k] == gs[k], k
        for k in EXACT + ("point", "pose", "fixed_pose", "match_train"):
            assert go[k].shape == gs[k].shape and np.array_equal(go[k].view(np.uint8), gs[k].view(np.uint8)), k
        for k, v in gs["summary"].items():
            assert go["summary"][k] == v, (k, go["summary"][k], v)
        assert Mo.trace() == Ms.trace()  # the last step's per-iteration records, bit for bit
    finally:
        Mo.close()
        if Ms is not None:
            Ms.close()
        for d in dev:
            for a in d[3:]:
                a.free()


def _dev_keyframes(ctx, seq, n):
    return [(k["pose"], k["Tcw"], len(k["x"]), ctx.to_device(A.u8(k["desc"])), ctx.to_device(A.f32(k["x"])),
             ctx.to_device(A.f32(k["y"])), ctx.to_device(A.f32(k["depth"]))) for k in seq["steps"][:n]]


def _bitwise_same(a, b, label):
    for k in ("t0", "points", "observations", "keypoints", "new_points", "new_observations", "matches"):
        assert a[k] == b[k], (label, k, a[k], b[k])
    for k in EXACT + ("point", "pose", "fixed_pose", "match_train"):
        assert a[k].shape == b[k].shape and np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), (label, k)
    for k, v in b["summary"].items():
        assert a["summary"][k] == v, (label, k, a["summary"][k], v)


def _group_vs_solo(ctx, seqs, n_steps, expect_fused, overlap=False):
    """maps stepped together (lorb_map_group, one ctx) vs the same maps stepped one by one
    (lorb_map_step_dev, a second set of maps): bit for bit after every step, LM traces included.
    overlap: the group's maps with lorb_map_set_overlap on (the keyframes are resident beforehand)"""
    from lorb_slam_amd.runtime import MapGroup
    fp = A.make_frame_params(synth.frame_params())
    devs = [_dev_keyframes(ctx, s, n_steps) for s in seqs]
    ctx.sync()
    Mg = [LocalMap(ctx, s["init"]) for s in seqs]
    Ms = [LocalMap(ctx, s["init"]) for s in seqs]
    for m in Mg:
        m.set_overlap(overlap)
    G = MapGroup(Mg)
    try:
        for t in range(n_steps):
            G.step_dev(fp, [d[t] for d in devs], OPT10)
            for m, d in zip(Ms, devs):
                m.step_dev(fp, *d[t], OPT10)
            for i, (a, b) in enumerate(zip(Mg, Ms)):
                _bitwise_same(a.read(), b.read(), f"map {i} step {t}")
                assert a.trace() == b.trace(), (i, t)
        info = G.info()
        assert info["maps"] == len(seqs) and info["plan_groups"] == (len(seqs) + 3) // 4, info
        assert info["fused_steps"] == (n_steps if expect_fused else 0), info
        return info
    finally:
        G.close()
        for m in Mg + Ms:
            m.close()
        for d in devs:
            for k in d:
                for a in k[3:]:
                    a.free()


@pytest.mark.parametrize("overlap", [False, True])
def test_local_mapping_group_bit_identical(ctx, overlap):
    """several windows stepped through ONE set of BA launches per step (the
    maps' device-built plans solved as a lorb_ba_group: every point-group, block and Cholesky kernel
    launched once for all of them).  Two C4 windows and a 24-keyframe one, 3 steps: each map equals
    the same map stepped alone, bit for bit (structure, poses, points, LM summary and per-iteration
    trace), and every group step ran fused; the solo chain itself is the oracle-checked one
    (test_local_mapping_chain_c4)."""
    seqs = [synth.mapping_sequence(seed=4, steps=3), synth.mapping_sequence(seed=21, steps=3),
            synth.mapping_sequence(seed=9, n_kf=24, n_fixed=3, n_new=90, obs_lens=(4, 5), steps=3, n_kps=800)]
    info = _group_vs_solo(ctx, seqs, 3, expect_fused=True, overlap=overlap)
    assert info["captures"] <= 3, info


def test_local_mapping_group_chunks_and_fallback(ctx):
    """Six small windows: two plan groups (4 + 2 maps).  With a 12-keyframe window among them (too
    narrow for the two-sided Cholesky) its plan group solves its members one by one; the results
    are bit-identical either way."""
    small = [synth.mapping_sequence(seed=30 + i, n_kf=24, n_fixed=3, n_new=90, obs_lens=(4, 5), steps=2, n_kps=800)
             for i in range(5)]
    tiny = synth.mapping_sequence(seed=9, n_kf=12, n_fixed=3, n_new=60, obs_lens=(4, 5), steps=2, n_kps=600)
    _group_vs_solo(ctx, small + [tiny], 2, expect_fused=False)


def test_local_mapping_group_step_error(ctx):
    """a group step where the second of three maps overflows its point capacity: that map is left as
    it was (as lorb_map_step_dev leaves it), the first completes its step (bit-identical to a solo
    step), the third is not stepped"""
    from lorb_slam_amd.runtime import MapGroup
    seq = synth.mapping_sequence(seed=5, n_kf=24, n_fixed=3, n_new=90, obs_lens=(4, 5), steps=2, n_kps=800)
    n_pts = len(seq["init"]["point_init"])
    fp = A.make_frame_params(synth.frame_params())
    dev = _dev_keyframes(ctx, seq, 2)
    ctx.sync()
    maps = [LocalMap(ctx, seq["init"]), LocalMap(ctx, seq["init"], max_points=n_pts + 5, max_keypoints=1024),
            LocalMap(ctx, seq["init"])]
    solo = LocalMap(ctx, seq["init"])
    G = MapGroup(maps)
    try:
        before = [m.read() for m in maps]
        with pytest.raises(LorbError, match="capacity"):
            G.step_dev(fp, [dev[0]] * 3, OPT10)
        solo.step_dev(fp, *dev[0], OPT10)
        _bitwise_same(maps[0].read(), solo.read(), "completed map")
        for i in (1, 2):
            after = maps[i].read()
            same_structure(after, before[i])
            for k in ("point", "pose", "fixed_pose"):
                assert np.array_equal(after[k], before[i][k]), (i, k)
        assert G.info()["fused_steps"] == 0
    finally:
        G.close()
        for m in maps + [solo]:
            m.close()
        for k in dev:
            for a in k[3:]:
                a.free()


def test_local_mapping_group_errors(ctx):
    """a group's maps share one context and appear once"""
    from lorb_slam_amd.runtime import Context, MapGroup
    seq = synth.mapping_sequence(seed=9, n_kf=12, n_fixed=3, n_new=60, obs_lens=(4, 5), steps=1, n_kps=600)
    c2 = Context(0)
    a, b, c = LocalMap(ctx, seq["init"]), LocalMap(ctx, seq["init"]), LocalMap(c2, seq["init"])
    try:
        with pytest.raises(LorbError, match="another context"):
            MapGroup([a, c])
        with pytest.raises(LorbError, match="twice"):
            MapGroup([a, b, a])
    finally:
        for m in (a, b, c):
            m.close()
        c2.close()
