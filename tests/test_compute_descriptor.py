"""MapPoint::ComputeDescriptor (src/map_point.cpp:69-129), SURVEY §8f row 4.

CPU: the oracle (sorted-row median, as the reference) against an independent numpy statement
(np.bitwise_count distance matrix + np.sort) on seeded, tie-heavy and edge-case lists.
GPU: liblorb.so bit-exact against the oracle (index and copied descriptor)."""
import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import synth


def numpy_ref(d_off, desc):
    out = []
    for p in range(len(d_off) - 1):
        D = desc[d_off[p]:d_off[p + 1]]
        n = len(D)
        if n == 0:
            out.append(-1)
            continue
        M = np.bitwise_count(D[:, None, :] ^ D[None, :, :]).sum(2)
        med = np.sort(M, axis=1)[:, int(0.5 * (n - 1))]
        out.append(int(np.argmin(med)))  # argmin = first index of the minimum
    return np.array(out, np.int32)


def lists(seed=5, n_points=400):
    """candidate lists: observations of a point are bit-flipped copies of one source descriptor
    (plus outliers), lengths 0..70 (empty, single, even/odd, > one wavefront)"""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 12, size=n_points)
    lens[:6] = [0, 1, 2, 3, 64, 70]
    descs = []
    for n in lens:
        src = synth.random_desc(rng, 1)
        d = synth.flip_bits(rng, np.repeat(src, n, 0), 24)
        k = n // 5
        if k:
            d[rng.choice(n, size=k, replace=False)] = synth.random_desc(rng, k)
        descs.append(d)
    d_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    desc = np.concatenate(descs) if descs else np.zeros((0, 32), np.uint8)
    return d_off, desc


def ties():
    """identical descriptors (every median ties) and two-element lists (median = 0 for both)"""
    rng = np.random.default_rng(9)
    a = synth.random_desc(rng, 1)
    d = [np.repeat(a, 5, 0), synth.random_desc(rng, 2), np.repeat(a, 4, 0)]
    d[2][3, 0] ^= 1
    d_off = np.concatenate([[0], np.cumsum([len(x) for x in d])]).astype(np.int32)
    return d_off, np.concatenate(d)


@pytest.mark.parametrize("case", ["lists", "ties"])
def test_oracle_vs_numpy(case):
    d_off, desc = lists() if case == "lists" else ties()
    assert np.array_equal(O.compute_descriptor(d_off, desc), numpy_ref(d_off, desc))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["lists", "ties"])
def test_gpu_compute_descriptor(ctx, case):
    d_off, desc = lists() if case == "lists" else ties()
    best, out = ctx.compute_descriptor(d_off, desc)
    ref = O.compute_descriptor(d_off, desc)
    assert np.array_equal(best, ref)
    for p in range(len(ref)):
        if ref[p] >= 0:
            assert np.array_equal(out[p], desc[d_off[p] + ref[p]])
        else:
            assert not out[p].any()
