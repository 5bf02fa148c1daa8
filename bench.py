#!/usr/bin/env python3
"""bench.py -- LORB_SLAM hot path on MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2]

Prints ONE JSON line on rank 0 (contract in the task description / DESIGN.md §Measurement).
Inputs are synthetic (lorb_slam_amd.synth, seeded per rank), generated on the host and
uploaded to HBM before the timed region.  Multi-GPU: launched by torch.distributed.run; each
rank processes its own independent windows / frame pairs (weak scaling, no data-path
collective); torch.distributed (gloo, CPU) only provides the barrier and the max-over-ranks of
the timing.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import synth  # noqa: E402
from lorb_slam_amd.runtime import Context, lib  # noqa: E402

INT32_VALU_PEAK = 256 * 4 * 32 * 2.4e9      # lane-ops/s: 256 CU x 4 SIMD32 x 2.4 GHz (MI355X_MICROARCH)
OPS_PER_PAIR = 16                             # 8 x v_xor_b32 + 8 x v_bcnt_u32_b32 per 256-bit pair


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist  # gloo on CPU: barrier + max-reduce of timings only
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


# ------------------------------------------------------------------------------------------
def workload_c2(ctx, args, rank):
    """BASELINE config 1: brute-force Hamming 2000x2000 random 256-bit + ratio test, batched
    over `pairs` independent frame pairs per GPU."""
    B = args.pairs
    qs, ts, ls = [], [], []
    for p in range(B):
        q, t, lev = synth.bf_problem(seed=1000 * rank + p, nq=2000, nt=2000, n_planted=1000, random_levels=True)
        qs.append(q); ts.append(t); ls.append(lev)
    q = np.concatenate(qs); t = np.concatenate(ts); lev = np.concatenate(ls)
    q_off = np.arange(B + 1, dtype=np.int32) * 2000
    t_off = np.arange(B + 1, dtype=np.int32) * 2000
    dq, dt, dl = ctx.to_device(q), ctx.to_device(t), ctx.to_device(lev)
    nq = len(q)
    outs = [ctx.empty(nq, np.int32) for _ in range(5)]
    acc = ctx.empty(nq, np.uint8)
    L = lib()

    def step():
        ctx.check(L.lorb_bf_top2_dev(ctx.handle, C.c_int32(B), dq.as_ptr(C.c_uint8), A.ptr(q_off, C.c_int32),
                                     dt.as_ptr(C.c_uint8), A.ptr(t_off, C.c_int32), dl.as_ptr(C.c_int32),
                                     *[o.as_ptr(C.c_int32) for o in outs], acc.as_ptr(C.c_uint8)), "bf_top2_dev")

    def check():
        return int(acc.numpy().sum())

    units = float(nq)                      # matches/s == queries resolved per second
    pairs = float(nq) * 2000.0
    return dict(step=step, check=check, units=units, pairs=pairs, kernel=A.__dict__.get("K", 0), kernel_id=0,
                config={"workload": "c2_bf_top2_ratio", "pairs_per_gpu": B, "nq": 2000, "nt": 2000},
                cpu=lambda: cpu_baseline_c2(qs[0], ts[0], ls[0]))


def cpu_baseline_c2(q, t, lev, budget_s=10.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: CPU restatement, timed as the reference-CPU baseline
    threads = max(1, min(16, os.cpu_count() or 1))
    O.bf_top2(q[:10], t, lev)  # build + warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        O.bf_top2(q, t, lev, threads=threads)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n * len(q) / dt, "unit": "matches/s", "cores": threads, "kind": "port",
            "sample": f"{n} x (2000x2000 bf top-2 + ratio test), oracle C restatement -O2, {threads} threads, {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2"])
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    D = Dist()
    ctx = Context(D.local_rank)
    wl = workload_c2(ctx, args, D.rank)
    for _ in range(args.warmup):
        wl["step"]()
    ctx.sync()
    L = lib()
    L.lorb_kernel_timing_enable(ctx.handle, 1)
    kms, kl = C.c_double(0), C.c_int(0)
    L.lorb_kernel_timing_read(ctx.handle, wl["kernel_id"], C.byref(kms), C.byref(kl))  # reset
    D.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl["step"]()
    ctx.sync()
    t1 = time.perf_counter()
    D.barrier()
    local = t1 - t0
    elapsed = D.max(local)
    L.lorb_kernel_timing_read(ctx.handle, wl["kernel_id"], C.byref(kms), C.byref(kl))
    L.lorb_kernel_timing_enable(ctx.handle, 0)
    checksum = wl["check"]()
    total_units = D.sum(wl["units"] * args.steps)
    value = total_units / elapsed
    avg_kernel_s = (kms.value / max(kl.value, 1)) * 1e-3
    launches_per_step = kl.value / args.steps
    ops_per_launch = wl["pairs"] * OPS_PER_PAIR / max(launches_per_step, 1)
    achieved = ops_per_launch / avg_kernel_s if avg_kernel_s > 0 else 0.0
    cpu = None
    if D.rank == 0 and not args.no_cpu_baseline:
        cpu = wl["cpu"]()
    if D.rank == 0:
        out = {
            "metric": "ORB matches/sec + local-BA iterations/sec (50 KF, 10k pts) at 1/2/4/8 MI355X",
            "value": value, "unit": "matches/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": dict(wl["config"], parallelism=f"replicas{D.world}"),
            "roofline": {"bound": "valu_int32", "achieved": achieved / 1e12, "peak": INT32_VALU_PEAK / 1e12,
                         "unit": "Tops/s", "frac": achieved / INT32_VALU_PEAK, "traffic": None,
                         "kernel": "k_bf_scan<TOP2>", "avg_kernel_us": avg_kernel_s * 1e6},
            "cpu_baseline": cpu, "checksum": checksum,
        }
        print(json.dumps(out))
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
