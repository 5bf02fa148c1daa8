"""CPU tests of the oracle's matcher restatement (test infrastructure) against independent
numpy computations and hand-built known-answer cases (the reference ships no fixtures)."""
import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import synth


def np_dist(q, t):
    return np.bitwise_count(q[:, None, :] ^ t[None, :, :]).sum(2).astype(np.int64)


def np_top2(D, lev):
    """src/matcher.cpp:289-311 restated over a distance matrix (numpy, independent of C)."""
    nq, nt = D.shape
    out = []
    for i in range(nq):
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for j in range(nt):
            d = D[i, j]
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, lev[j], j
            elif d < bd2:
                bl2, bd2 = lev[j], d
        acc = int(bd <= 100 and not (bl == bl2 and bd > 0.8 * bd2))
        out.append((bi, bd, bl, bd2, bl2, acc))
    return np.array(out)


def np_crosscheck(D):
    nq, nt = D.shape
    tidx, tdist = D.argmin(0), D.min(0)
    cc, dd = -np.ones(nq, int), np.full(nq, 1 << 30)
    for j in range(nt):
        i = tidx[j]
        if tdist[j] < dd[i]:
            dd[i], cc[i] = tdist[j], j
    m = cc >= 0
    if m.any():
        mn = dd[m].min()
        acc = m & (dd <= max(2 * mn, 30))
    else:
        acc = m
    return cc, np.where(m, dd, 0), np.where(acc, cc, -1)


def test_descriptor_distance_kat():
    z = np.zeros(32, np.uint8); f = np.full(32, 255, np.uint8)
    assert O.descriptor_distance(z, f) == 256
    assert O.descriptor_distance(z, z) == 0
    for bit in (0, 7, 8, 31, 32, 255):
        a = z.copy(); a[bit >> 3] ^= 1 << (bit & 7)
        assert O.descriptor_distance(z, a) == 1


def test_descriptor_distance_vs_numpy():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (2000, 32), dtype=np.uint8); b = rng.integers(0, 256, (2000, 32), dtype=np.uint8)
    ref = np.bitwise_count(a ^ b).sum(1)
    got = np.array([O.descriptor_distance(a[i], b[i]) for i in range(len(a))])
    assert (ref == got).all()


def test_ratio_and_filter_integer_identities():
    # bestDist > 0.8*bestDist2 (double) == 10*best > 8*second ; d > max(2m,30.0) == d > max(2m,30)
    for b in range(257):
        for s in range(257):
            assert (b > 0.8 * s) == (10 * b > 8 * s)
    for m in range(257):
        for d in range(257):
            assert (float(np.float32(d)) > max(2.0 * m, 30.0)) == (d > max(2 * m, 30))


@pytest.mark.parametrize("seed,random_levels", [(2, False), (7, True)])
def test_top2_vs_numpy(seed, random_levels):
    q, t, lev = synth.bf_problem(seed=seed, nq=120, nt=300, n_planted=80, random_levels=random_levels)
    r = O.bf_top2(q, t, lev)
    ref = np_top2(np_dist(q, t), lev)
    got = np.stack([r["best_idx"], r["best_dist"], r["best_level"], r["second_dist"], r["second_level"], r["accepted"]], 1)
    assert (got == ref).all()


def test_top2_ties_first_index_wins():
    q = np.zeros((1, 32), np.uint8)
    t = np.zeros((5, 32), np.uint8)
    for j, nb in enumerate([3, 1, 1, 2, 1]):
        for b in range(nb):
            t[j, b] = 1
    r = O.bf_top2(q, t, np.array([0, 4, 5, 0, 6], np.int32))
    assert r["best_idx"][0] == 1 and r["best_dist"][0] == 1 and r["best_level"][0] == 4
    assert r["second_dist"][0] == 1 and r["second_level"][0] == 5  # first remaining tie (j=2)


def test_top2_distance_256_never_enters():
    q = np.zeros((1, 32), np.uint8)
    t = np.full((3, 32), 255, np.uint8)
    r = O.bf_top2(q, t)
    assert r["best_idx"][0] == -1 and r["best_dist"][0] == 256 and r["second_level"][0] == -1


@pytest.mark.parametrize("seed", [2, 3])
def test_crosscheck_vs_numpy(seed):
    q, t, _ = synth.bf_problem(seed=seed, nq=150, nt=220, n_planted=100)
    r = O.bf_match(q, t)
    cc, dd, mt = np_crosscheck(np_dist(q, t))
    assert (r["cc_train"] == cc).all() and (r["cc_dist"] == dd).all() and (r["match_train"] == mt).all()
    assert r["n_matches"] == (mt >= 0).sum()


def test_crosscheck_asymmetric_kat():
    """Appendix C counter-example: t1's nearest query is q0, but q0's own nearest train (t0)
    is nearer to q1 -> OpenCV still returns (q0, t1), it is not a mutual-NN test."""
    def d(bits):
        a = np.zeros(32, np.uint8)
        for b in bits:
            a[b >> 3] |= 1 << (b & 7)
        return a
    q0 = d(range(0, 10)); q1 = d(range(0, 4))
    t0 = d(range(0, 5))          # d(q0,t0)=5, d(q1,t0)=1 -> nearest query q1
    t1 = d(list(range(0, 10)) + list(range(100, 107)))  # d(q0,t1)=7, d(q1,t1)=13 -> nearest q0
    r = O.bf_match(np.stack([q0, q1]), np.stack([t0, t1]))
    assert list(r["cc_train"]) == [1, 0]
    assert list(r["cc_dist"]) == [7, 1]


def test_crosscheck_empty_sets():
    q, t, _ = synth.bf_problem(seed=1, nq=10, nt=10)
    assert O.bf_match(q, t[:0])["n_matches"] == 0
    assert O.bf_match(q[:0], t)["n_matches"] == 0


def test_three_maxima_kat():
    h = np.zeros(30, int); h[3] = 10; h[7] = 5; h[9] = 5; h[11] = 1
    assert O.compute_three_maxima(h) == (3, 7, 9)
    h = np.zeros(30, int); h[3] = 100; h[7] = 9; h[9] = 20
    assert O.compute_three_maxima(h) == (3, 9, -1)  # 20 demotes 9 to third; 9 < 0.1*100 -> cut
    h = np.zeros(30, int)
    assert O.compute_three_maxima(h) == (-1, -1, -1)
    h = np.zeros(30, int); h[0] = 50; h[1] = 40; h[2] = 4
    assert O.compute_three_maxima(h) == (0, 1, -1)


def test_radius_by_viewing_cos():
    assert O.radius_by_viewing_cos(0.999) == 2.5
    assert O.radius_by_viewing_cos(0.998) == 2.5  # float(0.998) = 0.99800003 > 0.998 (double)
    assert O.radius_by_viewing_cos(0.99799) == 4.0
    assert O.radius_by_viewing_cos(0.5) == 4.0
