"""TEST INFRASTRUCTURE ONLY -- the chained LocalMapping step (include/lorb_c.h lorb_map_*) restated
on the CPU.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.

The step composes the oracle's restatements -- Matcher::SearchLocalPoints (or_bf_match,
src/matcher.cpp:319-366), Frame::UnprojectStereo (or_unproject_stereo, src/frame.cpp:335-356) and
BA::LocalPoseOptimization (or_ba_local, src/bundle_adjust.cpp:207-330) -- with the bookkeeping of
LocalMapping::ProcessNewFrames' disabled steps (src/local_mapping.cpp:55-76) written as plain numpy:
  1. a keypoint with a match adds an observation (point, keyframe, uv) to its map point
     (MapPoint::AddObservation, src/local_mapping.cpp:57-70);
  2. an unmatched keypoint with depth > 0 becomes a new map point (unprojected position, the
     keypoint's descriptor) observed by the keyframe;  1 and 2 append in keypoint order;
  3. the window slides by one keyframe (the sliding-window policy of DESIGN.md §5): points no window
     keyframe observes leave, observations by keyframes older than the F fixed ones are dropped,
     order is kept;
  observations are kept sorted by point, stably (a point's observations in the order they were
  added): the initial ones are sorted once, a step's new observations go after their point's
  earlier ones (the BA plan then needs no sort by point);
  4. LocalPoseOptimization of the window, float write-back (src/bundle_adjust.cpp:317-329).
Parity of the composed pieces is pinned where theirs is (oracle/lorb_oracle.h); the bookkeeping has
no reference counterpart to pin against (the reference's step is commented out).
"""
import numpy as np

import oracle as O


class MapOracle:
    def __init__(self, init, t0=0):
        """init: dict(pose_init W x 6 (keyframes t0..t0+W-1), fixed_pose F x 6 (t0-1..t0-F),
        point_init, point_desc, obs_point, obs_kf, obs_uv, intr)"""
        self.W, self.F = len(init["pose_init"]), len(init["fixed_pose"])
        self.intr = tuple(np.float32(v) for v in init["intr"])
        self.ring = {}
        for j in range(self.W):
            self.ring[t0 + j] = np.asarray(init["pose_init"][j], np.float32).copy()
        for j in range(self.F):
            self.ring[t0 - 1 - j] = np.asarray(init["fixed_pose"][j], np.float32).copy()
        self.point = np.asarray(init["point_init"], np.float32).reshape(-1, 3).copy()
        self.desc = np.asarray(init["point_desc"], np.uint8).reshape(-1, 32).copy()
        self.obs_point = np.asarray(init["obs_point"], np.int32).copy()
        self.obs_kf = np.asarray(init["obs_kf"], np.int32).copy()
        self.obs_uv = np.asarray(init["obs_uv"], np.float32).reshape(-1, 2).copy()
        self._sort_obs()
        self._slide(t0)

    def _sort_obs(self):
        o = np.argsort(self.obs_point, kind="stable")
        self.obs_point, self.obs_kf, self.obs_uv = self.obs_point[o], self.obs_kf[o], self.obs_uv[o]

    @classmethod
    def from_state(cls, st, intr):
        """from a LocalMap.read() (the device map's state)"""
        return cls(dict(pose_init=st["pose"], fixed_pose=st["fixed_pose"], point_init=st["point"],
                        point_desc=st["point_desc"], obs_point=st["obs_point"], obs_kf=st["obs_kf"],
                        obs_uv=st["obs_uv"], intr=intr), t0=st["t0"])

    def _slide(self, t0):
        keep_pt = np.zeros(len(self.point), bool)
        keep_pt[self.obs_point[self.obs_kf >= t0]] = True
        keep_obs = keep_pt[self.obs_point] & (self.obs_kf >= t0 - self.F)
        newid = np.cumsum(keep_pt) - 1
        self.point, self.desc = self.point[keep_pt], self.desc[keep_pt]
        self.obs_point = newid[self.obs_point[keep_obs]].astype(np.int32)
        self.obs_kf, self.obs_uv = self.obs_kf[keep_obs], self.obs_uv[keep_obs]
        kf = self.obs_kf
        self.obs_frame = np.where(kf >= t0, kf - t0, -1 - (t0 - 1 - kf)).astype(np.int32)
        self.t0 = t0
        self.ring = {k: v for k, v in self.ring.items() if k >= t0 - self.F}

    def window(self):
        return dict(pose_init=np.array([self.ring[self.t0 + j] for j in range(self.W)], np.float32),
                    fixed_pose=np.array([self.ring[self.t0 - 1 - j] for j in range(self.F)], np.float32).reshape(-1, 6),
                    point_init=self.point, obs_point=self.obs_point, obs_frame=self.obs_frame, obs_uv=self.obs_uv,
                    intr=self.intr)

    def step(self, fp, kf, opt):
        """one step with keyframe kf (synth.mapping_sequence()["steps"][i]); returns the matcher
        outputs and the BA's double-precision solution + summary"""
        n = len(kf["x"])
        t_new = self.t0 + self.W
        if len(self.point) > 0 and n > 0:
            m = O.bf_match(kf["desc"], self.desc)
            mt, nm = m["match_train"], m["n_matches"]
        else:
            mt, nm = np.full(n, -1, np.int32), 0
        xyz = O.unproject_stereo(fp, kf["Tcw"], kf["x"], kf["y"], kf["depth"])
        matched = mt >= 0
        new = ~matched & (np.asarray(kf["depth"], np.float32) > 0)
        sel = matched | new
        new_id = len(self.point) + np.cumsum(new) - 1
        obs_pt = np.where(matched, mt, new_id)[sel].astype(np.int32)
        self.point = np.concatenate([self.point, xyz[new].astype(np.float32)])
        self.desc = np.concatenate([self.desc, np.asarray(kf["desc"], np.uint8)[new]])
        uv = np.stack([np.asarray(kf["x"], np.float32), np.asarray(kf["y"], np.float32)], 1)[sel]
        self.obs_point = np.concatenate([self.obs_point, obs_pt])
        self.obs_kf = np.concatenate([self.obs_kf, np.full(int(sel.sum()), t_new, np.int32)])
        self.obs_uv = np.concatenate([self.obs_uv, uv])
        self.ring[t_new] = np.asarray(kf["pose"], np.float32).copy()
        self._sort_obs()
        self._slide(self.t0 + 1)
        poses, pts, summ, trace = O.ba_local_traced(self.window(), opt)
        for j in range(self.W):
            self.ring[self.t0 + j] = poses[j].astype(np.float32)
        self.point = pts.astype(np.float32)
        return dict(match_train=mt, n_matches=int(nm), new_points=int(new.sum()), new_observations=int(sel.sum()),
                    pose=poses, points=pts, summary=summ, trace=trace)

    def state(self):
        w = self.window()
        return dict(point=self.point, point_desc=self.desc, obs_point=self.obs_point, obs_kf=self.obs_kf,
                    obs_uv=self.obs_uv, obs_frame=self.obs_frame, pose=w["pose_init"], fixed_pose=w["fixed_pose"],
                    t0=self.t0, points=len(self.point), observations=len(self.obs_point))
