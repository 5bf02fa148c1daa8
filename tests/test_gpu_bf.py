"""GPU parity: brute-force Hamming kernels (liblorb.so) vs the oracle, bit-exact."""
import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import synth

pytestmark = pytest.mark.gpu


def _oracle_top2(q, t, lev):
    return O.bf_top2(q, t, lev)


@pytest.mark.parametrize("nq,nt,random_levels", [(2000, 2000, False), (2000, 2000, True), (300, 5000, True),
                                                  (1, 1, False), (257, 63, True), (5000, 129, False)])
def test_top2_single(ctx, nq, nt, random_levels):
    q, t, lev = synth.bf_problem(seed=nq + nt, nq=nq, nt=nt, n_planted=min(nq, nt) // 2, random_levels=random_levels)
    got, _ = ctx.bf_top2([q], [t], [lev])
    ref = _oracle_top2(q, t, lev)
    for k in ref:
        assert (got[k] == ref[k]).all(), k


@pytest.mark.parametrize("nt", [2, 3, 4, 5, 8, 11, 12, 13, 19, 28])
def test_top2_scan_remainders(ctx, nt):
    """Train counts around the scan loop's shape (two 4-descriptor steps per iteration, then one
    step, then single descriptors): every remainder path, bit-exact."""
    q, t, lev = synth.bf_problem(seed=700 + nt, nq=70, nt=nt, n_planted=min(70, nt) // 2, random_levels=True)
    got, _ = ctx.bf_top2([q], [t], [lev])
    ref = _oracle_top2(q, t, lev)
    for k in ref:
        assert (got[k] == ref[k]).all(), k
    got, _ = ctx.bf_match([q], [t])  # the top-1 scans (crossCheck, both directions)
    ref = O.bf_match(q, t)
    m = ref["cc_train"] >= 0
    assert (got["cc_train"] == ref["cc_train"]).all()
    assert (got["cc_dist"][m] == ref["cc_dist"][m]).all()
    assert (got["match_train"] == ref["match_train"]).all()
    assert got["n_matches"][0] == ref["n_matches"]


def test_top2_batched_ragged(ctx):
    rng = np.random.default_rng(11)
    qs, ts, ls = [], [], []
    for p in range(37):
        nq = int(rng.integers(0, 700)); nt = int(rng.integers(0, 900))
        q, t, lev = synth.bf_problem(seed=100 + p, nq=max(nq, 1), nt=max(nt, 1), n_planted=min(nq, nt) // 3,
                                     random_levels=True)
        qs.append(q[:nq]); ts.append(t[:nt]); ls.append(lev[:nt])
    got, q_off = ctx.bf_top2(qs, ts, ls)
    for p in range(len(qs)):
        ref = _oracle_top2(qs[p], ts[p], ls[p])
        for k in ref:
            assert (got[k][q_off[p]:q_off[p + 1]] == ref[k]).all(), (p, k)


def test_top2_ties_and_256(ctx):
    q = np.zeros((2, 32), np.uint8)
    t = np.zeros((6, 32), np.uint8)
    for j, nb in enumerate([3, 1, 1, 2, 1]):
        t[j, :nb] = 1
    t[5, :] = 255
    q[1, :] = 255; q[1, 0] = 0  # q1 vs t5 -> d=8 ; vs zeros-ish -> large
    lev = np.array([0, 4, 5, 0, 6, 2], np.int32)
    got, _ = ctx.bf_top2([q], [t], [lev])
    ref = O.bf_top2(q, t, lev)
    for k in ref:
        assert (got[k] == ref[k]).all(), k
    got, _ = ctx.bf_top2([np.zeros((1, 32), np.uint8)], [np.full((4, 32), 255, np.uint8)])
    assert got["best_idx"][0] == -1 and got["best_dist"][0] == 256


@pytest.mark.parametrize("nq,nt", [(2000, 2000), (500, 200), (2000, 10000), (1, 5), (7, 1)])
def test_crosscheck_single(ctx, nq, nt):
    q, t, _ = synth.bf_problem(seed=3 * nq + nt, nq=nq, nt=nt, n_planted=min(nq, nt) // 2)
    got, _ = ctx.bf_match([q], [t])
    ref = O.bf_match(q, t)
    m = ref["cc_train"] >= 0
    assert (got["cc_train"] == ref["cc_train"]).all()
    assert (got["cc_dist"][m] == ref["cc_dist"][m]).all()
    assert (got["match_train"] == ref["match_train"]).all()
    assert got["n_matches"][0] == ref["n_matches"]


def test_crosscheck_batched_with_empty(ctx):
    rng = np.random.default_rng(5)
    qs, ts = [], []
    for p in range(20):
        nq = int(rng.integers(0, 400)) if p % 5 else 0
        nt = int(rng.integers(0, 400)) if p % 7 else 0
        q, t, _ = synth.bf_problem(seed=p, nq=max(nq, 1), nt=max(nt, 1), n_planted=min(nq, nt) // 2)
        qs.append(q[:nq]); ts.append(t[:nt])
    got, q_off = ctx.bf_match(qs, ts)
    for p in range(len(qs)):
        ref = O.bf_match(qs[p], ts[p])
        sl = slice(q_off[p], q_off[p + 1])
        assert (got["cc_train"][sl] == ref["cc_train"]).all(), p
        assert (got["match_train"][sl] == ref["match_train"]).all(), p
        assert got["n_matches"][p] == ref["n_matches"], p
