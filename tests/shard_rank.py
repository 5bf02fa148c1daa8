"""One rank of the point-partitioned local BA for tests/test_gpu_shard.py.

    python tests/shard_rank.py RANK WORLD PORT OUT.npz

Builds the rank's shard of a synthetic window, joins a 2-rank host all-reduce over a local
socket (commutative ops, so both ranks hold bit-identical reduced values), runs the sharded
plan on GPU 0 (several ranks share the one GPU of the test box) and saves poses + its points."""
import os
import sys
from multiprocessing.connection import Client, Listener

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import shard, synth  # noqa: E402
from lorb_slam_amd.runtime import BAPlan, Comm, Context, LorbError  # noqa: E402

WINDOWS = [dict(seed=3, n_kf=12, n_pts=1500, n_fixed=2, fixed_obs_per_kf=150),
           dict(seed=7, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)]


def match_problems():
    """brute-force crossCheck problems: one with a planted majority, one ragged, one with no trains,
    one whose queries all fall on a single rank"""
    out = []
    for seed, nq, nt in ((21, 1500, 2000), (22, 333, 517), (23, 40, 0), (24, 1, 300)):
        q, t, _ = synth.bf_problem(seed=seed, nq=nq, nt=max(nt, 1), n_planted=min(nq, nt) // 2)
        out.append((q, t[:nt]))
    return out


def row_range(n, rank, world):
    return n * rank // world, n * (rank + 1) // world


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    assert world == 2
    if rank == 0:
        conn = Listener(("127.0.0.1", port), authkey=b"lorb").accept()
    else:
        import time
        t0 = time.time()
        while True:  # rank 0 may not be listening yet
            try:
                conn = Client(("127.0.0.1", port), authkey=b"lorb")
                break
            except ConnectionRefusedError:
                if time.time() - t0 > 60:
                    raise
                time.sleep(0.1)

    def allreduce(buf, op):
        conn.send_bytes(buf.tobytes())
        other = np.frombuffer(conn.recv_bytes(), dtype=np.float64)
        if op == 0:
            buf += other
        elif op == 1:
            np.maximum(buf, other, out=buf)
        else:
            np.minimum(buf, other, out=buf)

    ctx = Context(0)
    comm = Comm.host(ctx, world, rank, allreduce)
    res = {}
    # matcher: query rows split over the ranks, trains replicated
    probs = match_problems()
    ql, qb, tl = [], [], []
    for q, t in probs:
        a, b = row_range(len(q), rank, world)
        ql.append(q[a:b]); qb.append(a); tl.append(t)
    m = ctx.bf_match_sharded(comm, ql, qb, tl)
    for k, v in m.items():
        res[f"match_{k}"] = v
    wins = [synth.ba_window(**kw) for kw in WINDOWS]
    shards = [shard.shard_window(w, rank, world) for w in wins]
    for name, opt in (("default", A.LMOptions.default()),
                      ("ten", A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0,
                                                  gradient_tolerance=0.0, parameter_tolerance=0.0))):
        plan = BAPlan(ctx, shards, comm=comm)
        plan.solve(opt)
        P, X, S = plan.read()
        plan.close()
        for i in range(len(wins)):
            res[f"{name}_pose{i}"] = P[i]
            res[f"{name}_pts{i}"] = X[i]
            res[f"{name}_range{i}"] = np.array(shards[i]["point_range"])
            res[f"{name}_iters{i}"] = np.array([S[i]["iterations"], S[i]["successful_steps"]])
            res[f"{name}_cost{i}"] = np.array([S[i]["final_cost"]])
    # the device-built sharded plan (lorb_ba_plan_create_sharded_dev), one plan per window, built,
    # solved, rebuilt in place (collective update) and solved again
    from lorb_slam_amd.runtime import BAPlanDev
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    for i, sh in enumerate(shards):
        arrays = BAPlanDev.upload(ctx, sh, extra_points=11, extra_obs=97)
        plan = BAPlanDev(ctx, arrays, len(sh["pose_init"]), len(sh["fixed_pose"]), sh["intr"], comm=comm)
        plan.solve(opt)
        plan.update()
        plan.solve(opt)
        P, X, S = plan.read()
        res[f"dev_pose{i}"], res[f"dev_pts{i}"] = P[0], X[0]
        res[f"dev_iters{i}"] = np.array([S[0]["iterations"], S[0]["successful_steps"]])
        plan.close()
        for a in arrays.values():
            a.free()
    # a build failure on ONE rank is collective: the other rank's build reaches the exchange, and both
    # return the error (neither is left waiting); the plan then rebuilds and solves normally
    sh = shards[0]
    arrays = BAPlanDev.upload(ctx, sh, extra_points=11, extra_obs=97)
    plan = BAPlanDev(ctx, arrays, len(sh["pose_init"]), len(sh["fixed_pose"]), sh["intr"], comm=comm)
    over = dict(arrays)  # rank 1: a live observation count beyond its capacity (seen on the device)
    n_live = len(sh["obs_point"]) + (97 + 5 if rank == 1 else 0)
    over["n_obs"] = ctx.to_device(np.array([n_live], np.int32))
    errs = []
    try:
        plan.update(over)
        errs.append("")
    except LorbError as e:
        errs.append(str(e))
    over["n_obs"].free()
    plan.win = plan._window(arrays, sh["intr"])
    plan.win.n_poses += rank  # rank 1: a window shape that differs from the plan's (seen on the host)
    try:
        plan.update()
        errs.append("")
    except LorbError as e:
        errs.append(str(e))
    plan.win.n_poses -= rank
    plan.update()
    plan.solve(opt)
    P, X, S = plan.read()
    res["fail_msgs"] = np.array(errs)
    res["fail_pose"], res["fail_pts"] = P[0], X[0]
    res["fail_iters"] = np.array([S[0]["iterations"], S[0]["successful_steps"]])
    plan.close()
    for a in arrays.values():
        a.free()
    comm.close()
    ctx.close()
    np.savez(out, **res)
    conn.close()


if __name__ == "__main__":
    main()
