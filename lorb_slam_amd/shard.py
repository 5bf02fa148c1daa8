"""Point partition of a local-BA window over ranks ("one window point-partitioned
across GPUs").  Every rank keeps all window poses, fixed poses and intrinsics; points are split
into contiguous ranges balanced by observation count, and each point travels with ALL of its
observations, so the Schur elimination of a point is rank-local."""
import numpy as np


def point_ranges(win, world):
    """[start, stop) point range of every rank, balanced by observation count."""
    n = len(win["point_init"])
    cnt = np.bincount(np.asarray(win["obs_point"]), minlength=n).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def shard_window(win, rank, world):
    """This rank's shard: same poses, its point range (re-indexed from 0) and their observations,
    sorted by point (stably: a point's observations keep their relative order), so that the
    device-built plan takes its sorted path (k_db_sorted, no counting sort) every step."""
    a, b = point_ranges(win, world)[rank]
    op = np.asarray(win["obs_point"])
    sel = np.flatnonzero((op >= a) & (op < b))
    sel = sel[np.argsort(op[sel], kind="stable")]
    out = dict(win)
    out["point_init"] = np.ascontiguousarray(win["point_init"][a:b])
    out["obs_point"] = np.ascontiguousarray(op[sel] - a, dtype=np.int32)
    out["obs_frame"] = np.ascontiguousarray(np.asarray(win["obs_frame"])[sel], dtype=np.int32)
    out["obs_uv"] = np.ascontiguousarray(np.asarray(win["obs_uv"])[sel])
    out["point_range"] = (a, b)
    for k in ("true_points",):
        if k in win:
            out[k] = win[k][a:b]
    return out
