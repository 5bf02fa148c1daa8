"""Generate the committed golden fixtures under tests/golden/ (inputs + expected outputs, .npz).

The reference ships no golden vectors, known-answer tests or fixtures and cannot be built here
(SURVEY.md §8c), so these vectors are produced by the oracle (oracle/, the C restatement) and are
only written after the oracle agrees with an INDEPENDENT computation at generation time:
  * Hamming / crossCheck / top-2 + ratio test: numpy bitwise_count restatements
    (tests/test_oracle_match.py np_crosscheck / np_top2);
  * windowed search (a5): the pure-Python restatement tests/pyref.py;
  * BA: the oracle's LM (Ceres semantics); the fixture freezes it (parity unpinned vs Ceres).
The tests then hold both the oracle (CPU, `-m "not gpu"`) and liblorb.so (`-m gpu`) to them.

    python tools/make_golden.py            # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
import pyref  # noqa: E402
import golden_io  # noqa: E402
from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import synth  # noqa: E402
from test_oracle_match import np_crosscheck, np_top2  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def hamming():
    rng = np.random.default_rng(20261015)
    cases = []
    # edge cases: all-zero vs all-one, single-bit flips, ties (duplicate trains -> first wins)
    z = np.zeros((1, 32), np.uint8); f = np.full((1, 32), 255, np.uint8)
    q = np.concatenate([z, f, rng.integers(0, 256, (62, 32), dtype=np.uint8)])
    t = rng.integers(0, 256, (80, 32), dtype=np.uint8)
    t[3] = q[5]; t[4] = q[5]            # exact duplicates: crossCheck tie -> lowest train index
    t[10] = q[7]; t[10, 0] ^= 1         # distance 1
    t[11] = t[10]                       # duplicate train at distance 1
    lev = rng.integers(0, 8, 80).astype(np.int32)
    cases.append(("kat", q, t, lev))
    for name, nq, nt, planted in (("ragged", 37, 129, 20), ("medium", 500, 700, 300)):
        q, t, lev = synth.bf_problem(seed=nq * 7 + nt, nq=nq, nt=nt, n_planted=planted, random_levels=True)
        cases.append((name, q, t, lev))
    out = {}
    for name, q, t, lev in cases:
        D = np.bitwise_count(q[:, None, :] ^ t[None, :, :]).sum(2).astype(np.int64)
        m = O.bf_match(q, t)
        cc, dd, mt = np_crosscheck(D)
        assert np.array_equal(m["cc_train"], cc) and np.array_equal(m["match_train"], mt), name
        t2 = O.bf_top2(q, t, lev)
        ref = np_top2(D, lev)
        assert np.array_equal(t2["best_idx"], ref[:, 0]) and np.array_equal(t2["accepted"], ref[:, 5]), name
        extra = {"dist": D.astype(np.int32)} if name != "medium" else {}
        out[name] = dict(q=q, t=t, t_level=lev, **extra,
                         cc_train=m["cc_train"], cc_dist=m["cc_dist"], match_train=m["match_train"],
                         n_matches=m["n_matches"], **{k: v for k, v in t2.items()})
    golden_io.save(os.path.join(OUT, "hamming.npz"), out)
    print("hamming:", {k: int(v["n_matches"]) for k, v in out.items()})


def windows():
    out = {}
    pr = synth.local_points_problem(seed=11, n_kps=600, n_pts=800, n_true=400)
    a, n = O.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 1.0)
    ra, rn = pyref.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 1.0)
    assert np.array_equal(a, ra) and n == rn
    out["local"] = dict(inp=pr, th=1.0, assign=a, n=n)
    a3, n3 = O.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 3.0)
    ra, rn = pyref.search_by_projection_local(pr["fp"], pr["kps"], pr["slot_state"], pr["pts"], 3.0)
    assert np.array_equal(a3, ra) and n3 == rn
    out["local_th3"] = dict(assign=a3, n=n3)
    tf = synth.two_frames(seed=12, n_kps=400, n_shared=160, prefilled=30)
    fa = {}
    for th in (15.0, 30.0):
        a, n = O.search_by_projection_frame(tf["fp"], tf["cur_Tcw"], tf["cur_kps"], tf["slot_state"], tf["last"], th)
        fa[f"th{int(th)}"] = dict(assign=a, n=n)
    out["frame"] = dict(inp=tf, **fa)
    st = synth.local_mapping_step(seed=13, n_kf=8, n_pts=600, n_fixed=2, fixed_obs_per_kf=60, n_kps=300, n_reobs=150)
    xyz = O.unproject_stereo(synth.frame_params(), st["kf_Tcw"], st["kf_x"], st["kf_y"], st["kf_depth"])
    out["unproject"] = dict(Tcw=st["kf_Tcw"], x=st["kf_x"], y=st["kf_y"], depth=st["kf_depth"], xyz=xyz)
    golden_io.save(os.path.join(OUT, "windows.npz"), out)
    print("windows:", out["local"]["n"], out["local_th3"]["n"], {k: v["n"] for k, v in fa.items()})


def ba():
    out = {}
    opt = A.LMOptions.default()
    pb = synth.pose_only_batch(seed=21, n_frames=3, n_res=120)
    pose, T, summ = O.ba_pose_only(pb, opt)
    out["pose_only"] = dict(inp=pb, pose=pose, Tcw=T, iterations=np.array([s["iterations"] for s in summ]),
                            final_cost=np.array([s["final_cost"] for s in summ]))
    wins = [synth.ba_window(seed=22 + i, n_kf=6, n_pts=300, n_fixed=2, fixed_obs_per_kf=40) for i in range(2)]
    poses, pts, summ = O.ba_local(wins, opt)
    out["local"] = dict(inp=wins, poses=poses, points=pts,
                        iterations=np.array([s["iterations"] for s in summ]),
                        final_cost=np.array([s["final_cost"] for s in summ]),
                        initial_cost=np.array([s["initial_cost"] for s in summ]))
    golden_io.save(os.path.join(OUT, "ba.npz"), out)
    print("ba:", out["local"]["iterations"], out["local"]["final_cost"], out["pose_only"]["iterations"])


REF = os.environ.get("LORB_REFERENCE", "/root/reference")


def orb_pattern():
    """bit_pattern_31_ (src/ORBextractor.cpp:152-410, the 256 ORB test pairs the reference's
    ORBextractor passes to computeOrbDescriptor), read from the reference tree as data."""
    import re
    src = open(os.path.join(REF, "src", "ORBextractor.cpp")).read()
    body = src[src.index("bit_pattern_31_[256*4]"):]
    body = body[body.index("{") + 1:body.index("};")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    vals = np.array([int(v) for v in body.replace("\n", " ").split(",") if v.strip()], np.int32)
    assert vals.shape == (1024,) and vals.min() >= -13 and vals.max() <= 12
    return vals


def orb():
    """The whole ORBextractor::operator() on a 752 x 480 scene at 1000 and 2000 features, with the
    reference's own bit_pattern_31_.  The oracle's keypoints are checked at generation time against
    the independent Python restatement (tests/pyref.py: cells, numpy FAST, list-based
    DistributeOctTree) and its descriptors against pyref.orb_describe (libm cosf)."""
    pattern = orb_pattern()
    img = synth.orb_scene(seed=91)
    sf = synth.scale_factors()
    out = {"pattern": pattern, "image": img}
    for nfeat in (1000, 2000):
        nd = O.orb_features_per_level(nfeat)
        e = O.orb_extract(img, nd, sf, pattern)
        pyr = O.orb_pyramid(img, sf)
        lo = e["level_off"]
        for l in range(8):
            kx, ky, kr = [], [], []
            for (ix, iy, w, h), (rx, ry) in zip(pyref.orb_cells(*pyr[l].shape), pyref_cell_offsets(*pyr[l].shape)):
                if w <= 0:
                    continue
                cell = pyr[l][iy:iy + h, ix:ix + w]
                fx, fy, fr = pyref.fast(cell, 20)
                if len(fx) == 0:
                    fx, fy, fr = pyref.fast(cell, 7)
                kx += list(fx + rx); ky += list(fy + ry); kr += list(fr)
            keep = pyref.distribute_octree(kx, ky, kr, 16, pyr[l].shape[1] - 16, 16, pyr[l].shape[0] - 16, nd[l])
            s = sf[l] if l else np.float32(1)
            sl = slice(lo[l], lo[l + 1])
            for key, v in (("x", kx), ("y", ky)):
                g = np.asarray(v, np.float32)[keep] + np.float32(16)
                g = g * s if l else g
                assert np.array_equal(e[key][sl], np.asarray(g, np.float32)), (nfeat, l, key)
            # response = the FAST score, octave = the level, size = PATCH_SIZE * scale truncated to
            # int (src/ORBextractor.cpp:878-882), all independent of the oracle
            assert np.array_equal(e["response"][sl], np.asarray(kr, np.float32)[keep]), (nfeat, l, "response")
            assert np.all(e["octave"][sl] == l), (nfeat, l, "octave")
            assert np.all(e["size"][sl] == np.float32(int(np.float32(31) * np.float32(sf[l])))), (nfeat, l, "size")
        d = O.orb_detect(pyr, nd, sf)
        ang, desc = pyref.orb_describe(pyr, d["x"], d["y"], d["octave"], pattern)
        assert np.array_equal(ang, e["angle"]) and np.array_equal(desc, e["desc"]), nfeat
        out[f"n{nfeat}"] = dict(n_desired=nd, **{k: v for k, v in e.items()})
    golden_io.save(os.path.join(OUT, "orb.npz"), out)
    print("orb:", {k: len(v["x"]) for k, v in out.items() if k.startswith("n")})


def pyref_cell_offsets(rows, cols):
    """(j wCell, i hCell) of every cell: the offset ComputeKeyPointsOctTree adds to the FAST
    coordinates (src/ORBextractor.cpp:865-866)."""
    import math
    width, height = np.float32(cols - 32), np.float32(rows - 32)
    nc, nr = int(width / np.float32(30)), int(height / np.float32(30))
    wc, hc = int(math.ceil(np.float32(width / np.float32(nc)))), int(math.ceil(np.float32(height / np.float32(nr))))
    return [(j * wc, i * hc) for i in range(nr) for j in range(nc)]


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    O.build()
    hamming()
    windows()
    ba()
    orb()
