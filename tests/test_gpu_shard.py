"""GPU: point-partitioned local BA through lorb_ba_plan_create_sharded.

* world 1 over RCCL (the communicator, the captured exchanges) == the unsharded plan;
* world 2, two processes sharing the test box's GPU, host all-reduce transport: poses and each
  rank's points == the unsharded solve within the north_star tolerance (1e-5 relative; the
  exchange only reorders sums, so the agreement is ~1e-10 in practice), same iteration counts."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from lorb_slam_amd import _abi as A
from lorb_slam_amd import synth

pytestmark = pytest.mark.gpu
RTOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import shard_rank  # noqa: E402


def close(a, b, rtol=RTOL):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(b), 1.0))


OPTS = {"default": A.LMOptions.default(),
        "ten": A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                                   parameter_tolerance=0.0)}


def test_sharded_rccl_world1_matches_unsharded(ctx):
    from lorb_slam_amd.runtime import BAPlan, Comm, unique_id
    wins = [synth.ba_window(**kw) for kw in shard_rank.WINDOWS]
    comm = Comm.rccl(ctx, 1, 0, unique_id())
    try:
        for opt in OPTS.values():
            ref = BAPlan(ctx, wins); ref.solve(opt); Pr, Xr, Sr = ref.read(); ref.close()
            pl = BAPlan(ctx, wins, comm=comm); pl.solve(opt); pl.solve(opt); Ps, Xs, Ss = pl.read(); pl.close()
            for i in range(len(wins)):
                assert close(Ps[i], Pr[i], 1e-9) and close(Xs[i], Xr[i], 1e-9)
                assert Ss[i]["iterations"] == Sr[i]["iterations"]
    finally:
        comm.close()


def test_sharded_two_ranks_host_transport(ctx, tmp_path):
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    outs = [str(tmp_path / f"r{r}.npz") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "shard_rank.py"), str(r), "2", str(port), outs[r]])
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    R = [np.load(o) for o in outs]
    # matcher rows: bit-exact vs the unsharded kernel (and the oracle)
    probs = shard_rank.match_problems()
    ref, _ = ctx.bf_match([q for q, _ in probs], [t for _, t in probs])
    def gather(k):  # rank r holds rows row_range(nq_p, r, 2) of every problem p, problems concatenated
        parts, off = [[], []], [0, 0]
        for q, _ in probs:
            for r in range(2):
                a, b = shard_rank.row_range(len(q), r, 2)
                parts[r].append(R[r][f"match_{k}"][off[r]:off[r] + b - a]); off[r] += b - a
        return np.concatenate([np.concatenate([parts[0][p], parts[1][p]]) for p in range(len(probs))])
    for k in ("cc_train", "match_train"):
        assert np.array_equal(gather(k), ref[k]), k
    has = ref["cc_train"] >= 0
    assert np.array_equal(gather("cc_dist")[has], ref["cc_dist"][has])
    assert np.array_equal(R[0]["match_n_matches"], ref["n_matches"]) and np.array_equal(R[1]["match_n_matches"], ref["n_matches"])
    for (q, t), n in zip(probs, ref["n_matches"]):
        assert O.bf_match(q, t)["n_matches"] == n
    wins = [synth.ba_window(**kw) for kw in shard_rank.WINDOWS]
    for name, opt in OPTS.items():
        Pg, Xg, Sg = ctx.ba_local(wins, opt)
        Po, Xo, So = O.ba_local(wins, opt)
        for i in range(len(wins)):
            # poses are replicated bit-identically on both ranks
            assert np.array_equal(R[0][f"{name}_pose{i}"], R[1][f"{name}_pose{i}"])
            assert close(R[0][f"{name}_pose{i}"], Pg[i]) and close(R[0][f"{name}_pose{i}"], Po[i])
            X = np.zeros_like(Xg[i])
            for r in range(2):
                a, b = R[r][f"{name}_range{i}"]
                X[a:b] = R[r][f"{name}_pts{i}"]
            assert close(X, Xg[i]) and close(X, Xo[i])
            assert list(R[0][f"{name}_iters{i}"]) == [Sg[i]["iterations"], Sg[i]["successful_steps"]]
    # the device-built sharded plans (10 iterations, tolerances 0) against the unsharded solve
    opt = OPTS["ten"]
    Pg, Xg, Sg = ctx.ba_local(wins, opt)
    for i in range(len(wins)):
        assert np.array_equal(R[0][f"dev_pose{i}"], R[1][f"dev_pose{i}"])
        assert close(R[0][f"dev_pose{i}"], Pg[i])
        X = np.zeros_like(Xg[i])
        for r in range(2):
            a, b = R[r][f"ten_range{i}"]
            X[a:b] = R[r][f"dev_pts{i}"]
        assert close(X, Xg[i])
        assert R[0][f"dev_iters{i}"][0] == Sg[i]["iterations"]
    # one rank over its capacity, then one rank with a wrong shape: both ranks return each error
    for r in range(2):
        m = list(R[r]["fail_msgs"])
        assert len(m) == 2 and all(m), (r, m)
        assert "capacity" in m[0], (r, m[0])
        assert "shape" in m[1] and ("this rank" if r == 1 else "another rank") in m[1], (r, m[1])
    # ... and the plan rebuilds and solves as before
    assert np.array_equal(R[0]["fail_pose"], R[1]["fail_pose"])
    assert close(R[0]["fail_pose"], R[0]["dev_pose0"], 1e-9)
    assert list(R[0]["fail_iters"]) == list(R[0]["dev_iters0"])


def test_sharded_dev_rccl_world1(ctx):
    """the device-built sharded plan at world 1 over RCCL equals the unsharded device-built plan"""
    from lorb_slam_amd.runtime import BAPlanDev, Comm, unique_id
    w = synth.ba_window(**shard_rank.WINDOWS[1])
    comm = Comm.rccl(ctx, 1, 0, unique_id())
    arrays = BAPlanDev.upload(ctx, w, extra_points=5, extra_obs=50)
    try:
        opt = OPTS["ten"]
        ref = BAPlanDev(ctx, arrays, len(w["pose_init"]), len(w["fixed_pose"]), w["intr"])
        ref.solve(opt); Pr, Xr, Sr = ref.read(); ref.close()
        pl = BAPlanDev(ctx, arrays, len(w["pose_init"]), len(w["fixed_pose"]), w["intr"], comm=comm)
        pl.solve(opt); pl.update(); pl.solve(opt); Ps, Xs, Ss = pl.read(); pl.close()
        assert close(Ps[0], Pr[0], 1e-9) and close(Xs[0], Xr[0], 1e-9)
        assert Ss[0]["iterations"] == Sr[0]["iterations"]
    finally:
        comm.close()
        for a in arrays.values():
            a.free()
