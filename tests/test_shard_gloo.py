"""CPU, world_size 2 over torch.distributed gloo: the point-partitioned local BA (the N>1 path,
SURVEY §8e) restated in the oracle with the GPU path's three exchanges per LM iteration, each an
all_reduce over gloo.  Poses and the gathered points must equal the single-process solve (the
exchange only reorders sums; tolerance 1e-9 relative), with the same iteration counts."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [dict(seed=3, n_kf=6, n_pts=300, n_fixed=2, fixed_obs_per_kf=60),
         dict(seed=5, n_kf=12, n_pts=900, n_fixed=2, fixed_obs_per_kf=120)]


def _rank(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch

    import oracle as O
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import shard, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ops = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MAX, 2: dist.ReduceOp.MIN}

    def allreduce(buf, op):
        t = torch.from_numpy(buf)  # shares memory with the oracle's buffer
        dist.all_reduce(t, op=ops[op])

    wins = [synth.ba_window(**kw) for kw in CASES]
    shards = [shard.shard_window(w, rank, world) for w in wins]
    res = {}
    for name, opt in (("default", A.LMOptions.default()),
                      ("ten", A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0,
                                                  gradient_tolerance=0.0, parameter_tolerance=0.0))):
        P, X, S = O.ba_local_sharded(shards, rank, allreduce, opt)
        for i in range(len(wins)):
            res[f"{name}_pose{i}"] = P[i]; res[f"{name}_pts{i}"] = X[i]
            res[f"{name}_range{i}"] = np.array(shards[i]["point_range"])
            res[f"{name}_iters{i}"] = np.array([S[i]["iterations"], S[i]["successful_steps"]])
    dist.destroy_process_group()
    np.savez(out.format(rank), **res)


@pytest.mark.parametrize("world", [2])
def test_sharded_oracle_over_gloo_matches_single_process(world, tmp_path):
    import oracle as O
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    out = str(tmp_path / "r{}.npz")
    mp.start_processes(_rank, args=(world, port, out), nprocs=world, join=True, start_method="spawn")
    R = [np.load(out.format(r)) for r in range(world)]
    wins = [synth.ba_window(**kw) for kw in CASES]
    for name, opt in (("default", A.LMOptions.default()),
                      ("ten", A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0,
                                                  gradient_tolerance=0.0, parameter_tolerance=0.0))):
        Po, Xo, So = O.ba_local(wins, opt)
        for i in range(len(wins)):
            for r in range(world):
                assert np.array_equal(R[r][f"{name}_pose{i}"], R[0][f"{name}_pose{i}"])
                assert list(R[r][f"{name}_iters{i}"]) == [So[i]["iterations"], So[i]["successful_steps"]]
            tol = 1e-9 * np.maximum(np.abs(Po[i]), 1.0)
            assert np.all(np.abs(R[0][f"{name}_pose{i}"] - Po[i]) <= tol)
            X = np.zeros_like(Xo[i])
            for r in range(world):
                a, b = R[r][f"{name}_range{i}"]
                X[a:b] = R[r][f"{name}_pts{i}"]
            assert np.all(np.abs(X - Xo[i]) <= 1e-9 * np.maximum(np.abs(Xo[i]), 1.0))
