"""CPU: the chained LocalMapping step's restatement (oracle/oracle_map.py) on a small keyframe
stream -- bookkeeping invariants and the synthetic ground truth (every re-observation keypoint
matches its own map point, every new-point keypoint creates one)."""
import numpy as np

from lorb_slam_amd import _abi as A
from lorb_slam_amd import synth
from oracle_map import MapOracle

OPT = A.LMOptions.default(max_num_iterations=5, function_tolerance=0.0, gradient_tolerance=0.0,
                          parameter_tolerance=0.0)


def small_sequence(steps=3):
    return synth.mapping_sequence(seed=7, n_kf=8, n_fixed=2, n_new=24, obs_lens=(3, 4), steps=steps, n_kps=160,
                                  max_flips=8)


def check_invariants(m):
    W, F, t0 = m.W, m.F, m.t0
    P, K = len(m.point), len(m.obs_point)
    assert len(m.desc) == P and len(m.obs_kf) == K and len(m.obs_uv) == K
    assert np.all((m.obs_point >= 0) & (m.obs_point < P))
    assert np.all((m.obs_kf >= t0 - F) & (m.obs_kf < t0 + W))
    # every point is seen by a window keyframe; no point twice by one keyframe
    assert np.array_equal(np.unique(m.obs_point[m.obs_kf >= t0]), np.arange(P))
    pairs = m.obs_point.astype(np.int64) * 1_000_000 + (m.obs_kf - t0 + F)
    assert len(np.unique(pairs)) == K
    # observations sorted by point (stable), the order the device map keeps
    assert np.all(np.diff(m.obs_point) >= 0)
    fr = m.obs_frame
    assert np.array_equal(fr >= 0, m.obs_kf >= t0)
    assert np.array_equal(np.where(fr >= 0, t0 + fr, t0 - 1 - (-1 - fr)), m.obs_kf)


def test_map_oracle_chained_steps():
    seq = small_sequence()
    fp = synth.frame_params()
    m = MapOracle(seq["init"])
    check_invariants(m)
    assert m.t0 == 0 and len(m.point) == len(seq["init"]["point_init"])
    for i, kf in enumerate(seq["steps"]):
        P0, d0 = len(m.point), m.desc.copy()
        r = m.step(fp, kf, OPT)
        check_invariants(m)
        assert m.t0 == i + 1
        # ground truth: distractors (random descriptors) never pass crossCheck + minDist, every
        # re-observation (<= 8 flipped bits) matches its own point, every new-point keypoint is new
        mt = r["match_train"]
        dist_ok = np.array([np.unpackbits(np.bitwise_xor(kf["desc"][q], d0[t])).sum() for q, t in enumerate(mt) if t >= 0])
        assert np.all(dist_ok <= 8)
        assert r["n_matches"] == kf["n_reobs"] and (mt >= 0).sum() == kf["n_reobs"]
        assert r["new_points"] == kf["n_new"]
        assert r["new_observations"] == kf["n_reobs"] + kf["n_new"]
        assert P0 > 0
        s = r["summary"]
        assert s["iterations"] == OPT.max_num_iterations and s["final_cost"] < s["initial_cost"]


def test_map_oracle_from_state_round_trip():
    seq = small_sequence(steps=1)
    m = MapOracle(seq["init"])
    m.step(synth.frame_params(), seq["steps"][0], OPT)
    st = m.state()
    m2 = MapOracle.from_state(st, seq["init"]["intr"])
    for k in ("point", "point_desc", "obs_point", "obs_kf", "obs_uv", "obs_frame", "pose", "fixed_pose"):
        assert np.array_equal(st[k], m2.state()[k]), k
    assert m2.t0 == m.t0


def test_map_oracle_empty_and_depthless_keyframes():
    seq = small_sequence(steps=1)
    fp = synth.frame_params()
    m = MapOracle(seq["init"])
    kf = dict(seq["steps"][0])
    # no keypoints: the window still slides (the oldest keyframe's points may leave) and BA runs
    empty = dict(kf, x=kf["x"][:0], y=kf["y"][:0], desc=kf["desc"][:0], depth=kf["depth"][:0])
    r = m.step(fp, empty, OPT)
    check_invariants(m)
    assert r["n_matches"] == 0 and r["new_points"] == 0
    # no stereo depth anywhere: matches only
    m2 = MapOracle(seq["init"])
    r = m2.step(fp, dict(kf, depth=np.full_like(kf["depth"], -1.0)), OPT)
    check_invariants(m2)
    assert r["new_points"] == 0 and r["new_observations"] == r["n_matches"]
