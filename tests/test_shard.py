"""CPU: the point partition used by the sharded local BA (lorb_slam_amd/shard.py)."""
import numpy as np
import pytest

from lorb_slam_amd import shard, synth


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_covers_points_once_and_keeps_observations(world):
    w = synth.ba_window(seed=11, n_kf=10, n_pts=900, n_fixed=2, fixed_obs_per_kf=90)
    shards = [shard.shard_window(w, r, world) for r in range(world)]
    ranges = [s["point_range"] for s in shards]
    assert ranges[0][0] == 0 and ranges[-1][1] == len(w["point_init"])
    assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
    assert sum(len(s["obs_point"]) for s in shards) == len(w["obs_point"])
    for s in shards:
        a, b = s["point_range"]
        assert np.array_equal(s["point_init"], w["point_init"][a:b])
        assert s["obs_point"].min(initial=0) >= 0 and s["obs_point"].max(initial=-1) < b - a
        assert np.array_equal(s["pose_init"], w["pose_init"]) and np.array_equal(s["fixed_pose"], w["fixed_pose"])
        # the shard's observations are the point range's, sorted by point, stably (a point's
        # observations keep their relative order): what the device plan's sorted path takes
        sel = np.flatnonzero((w["obs_point"] >= a) & (w["obs_point"] < b))
        sel = sel[np.argsort(w["obs_point"][sel], kind="stable")]
        assert np.all(np.diff(s["obs_point"]) >= 0)
        assert np.array_equal(s["obs_point"], w["obs_point"][sel] - a)
        assert np.array_equal(s["obs_frame"], w["obs_frame"][sel]) and np.array_equal(s["obs_uv"], w["obs_uv"][sel])
    if world > 1:
        nobs = [len(s["obs_point"]) for s in shards]
        assert max(nobs) - min(nobs) <= 2 * 16  # balanced to within a couple of points' observations
