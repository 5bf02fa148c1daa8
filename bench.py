#!/usr/bin/env python3
"""bench.py -- LORB_SLAM matcher + local-BA hot path on MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2] [--windows W]

Default workload (c4, BASELINE config "full local_mapping step -- match + triangulate + BA on a
50-KF / 10k-point sliding window"): per GPU and per step, for each of `--windows` independent
windows (default 1, i.e. C4 at N=1 and C5 -- one window per GPU -- at N=8):
  1. brute-force Hamming + OpenCV crossCheck + minDist filter of the new keyframe's 2,000
     descriptors against the window's 10,000 map-point descriptors (Matcher::SearchLocalPoints),
  2. stereo unprojection of the new keyframe's keypoints (Frame::UnprojectStereo),
  3. 10 Levenberg-Marquardt iterations of BA::LocalPoseOptimization on the window
     (50 optimised KFs + 5 fixed, 10,000 points, 77,000 observations), tolerances 0.
The window's observation structure (CSR, Schur block-pair lists) is built once per window
outside the timed region (reported as plan_build_ms).  `value` = LM iterations/s over all GPUs;
`matches_per_sec` = keyframe descriptors resolved per second in the same steps.

Inputs are synthetic (lorb_slam_amd.synth, seeded per rank) and resident in HBM before the
timed region.  Multi-GPU: launched by torch.distributed.run; each rank owns its own windows
(weak scaling, no data-path collective); torch.distributed (gloo, CPU) only provides the barrier
and the max-over-ranks of the timing.
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
from lorb_slam_amd.runtime import BAPlan, Context, device_count, lib  # noqa: E402

CLOCK = 2.4e9
INT32_VALU_PEAK = 256 * 4 * 32 * CLOCK      # lane-ops/s: 256 CU x 4 SIMD32 (MI355X_MICROARCH)
FP64_PEAK = 78.6e12                          # FP64 vector/matrix dense, MI355X spec
HBM_PEAK = 8.0e12                            # HBM3E spec (MI355X_MICROARCH)
OPS_PER_PAIR = 16                            # 8 x v_xor_b32 + 8 x v_bcnt_u32_b32 per 256-bit pair
# the Cholesky id covers three kernels chosen by band shape; C3/C4/C5 windows
# (band 47, n >= 128) run the two-sided k_ba_chol_2s
K_NAMES = {0: "k_bf_scan<top2>", 1: "k_bf_scan<top1>", 2: "k_ba_schur", 3: "k_ba_lin", 4: "k_ba_chol_2s"}
# rocprofv3 short names (tools/pmc_traffic.py) of the same kernels, for the PMC traffic lookup
K_PROF = {0: "k_bf_scan", 1: "k_bf_scan", 2: "k_ba_schur", 3: "k_ba_lin", 4: "k_ba_chol_2s"}
TRAFFIC = os.path.join(ROOT, "profiles", "r01", "traffic.json")
METRIC = "ORB matches/sec + local-BA iterations/sec (50 KF, 10k pts) at 1/2/4/8 MI355X"


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist  # gloo on CPU: barrier + reductions of timings only
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def reduce(self, v, op):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def broadcast_bytes(self, b):
        """rank 0's bytes to every rank (the RCCL unique id), over gloo"""
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def kernel_times(ctx, ids):
    L = lib()
    out = {}
    for k in ids:
        ms, n = C.c_double(0), C.c_int(0)
        L.lorb_kernel_timing_read(ctx.handle, k, C.byref(ms), C.byref(n))
        out[k] = (ms.value, n.value)
    return out


# ------------------------------------------------------------------------------------------
def workload_c4(ctx, args, rank):
    W = args.windows
    steps = [synth.local_mapping_step(seed=4 + 1009 * rank + 17 * i) for i in range(W)]
    wins = [s["window"] for s in steps]
    t0 = time.perf_counter()
    plan = BAPlan(ctx, wins)
    plan_ms = (time.perf_counter() - t0) * 1e3
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    nq, nt = len(steps[0]["kf_desc"]), len(steps[0]["mp_desc"])
    dq = ctx.to_device(np.concatenate([s["kf_desc"] for s in steps]))
    dt = ctx.to_device(np.concatenate([s["mp_desc"] for s in steps]))
    q_off = np.arange(W + 1, dtype=np.int32) * nq
    t_off = np.arange(W + 1, dtype=np.int32) * nt
    cc_t, cc_d, mt = (ctx.empty(W * nq, np.int32) for _ in range(3))
    nm = ctx.empty(W, np.int32)
    dx = [ctx.to_device(s["kf_x"]) for s in steps]
    dy = [ctx.to_device(s["kf_y"]) for s in steps]
    dd = [ctx.to_device(s["kf_depth"]) for s in steps]
    dxyz = [ctx.empty((nq, 3), np.float32) for _ in steps]
    fp = A.make_frame_params(synth.frame_params())
    Ts = [A.f32(s["kf_Tcw"]).reshape(16) for s in steps]
    L = lib()

    def step():
        ctx.check(L.lorb_bf_match_dev(ctx.handle, C.c_int32(W), dq.as_ptr(C.c_uint8), A.ptr(q_off, C.c_int32),
                                      dt.as_ptr(C.c_uint8), A.ptr(t_off, C.c_int32), cc_t.as_ptr(C.c_int32),
                                      cc_d.as_ptr(C.c_int32), mt.as_ptr(C.c_int32), nm.as_ptr(C.c_int32)),
                  "lorb_bf_match_dev")
        for i in range(W):
            ctx.check(L.lorb_unproject_stereo_dev(ctx.handle, C.byref(fp), A.ptr(Ts[i], C.c_float), C.c_int32(nq),
                                                  dx[i].as_ptr(C.c_float), dy[i].as_ptr(C.c_float),
                                                  dd[i].as_ptr(C.c_float), dxyz[i].as_ptr(C.c_float)),
                      "lorb_unproject_stereo_dev")
        plan.solve(opt)

    def check():
        n = nm.numpy()
        _, _, summ = plan.read()
        return {"n_matches": [int(v) for v in n], "ba_final_cost": [s["final_cost"] for s in summ],
                "ba_iterations": [s["iterations"] for s in summ]}

    # algorithmic work per step: matcher pairs, BA FP64 flops per LM iteration
    pairs = float(W) * nq * nt
    n_obs = sum(len(w["obs_point"]) for w in wins)
    n_pts = sum(len(w["point_init"]) for w in wins)
    F = len(wins[0]["pose_init"])
    kp = np.bincount(wins[0]["obs_point"][wins[0]["obs_frame"] >= 0])
    pt_flops = float(np.sum(60 + 108 * kp + 108 * kp * (kp + 1)))
    it_flops = W * (420.0 * n_obs / W + pt_flops + (6 * F) ** 3 / 3 + 4 * (6 * F) ** 2)
    # per-launch algorithmic work of each BA kernel (all windows of the step); DESIGN.md §Roofline
    pair_cnt = 0
    for w in wins:
        m = w["obs_frame"] >= 0
        k = np.bincount(w["obs_point"][m], minlength=len(w["point_init"]))
        pair_cnt += int(np.sum(k * (k + 1) // 2))
    opt_obs = sum(int((w["obs_frame"] >= 0).sum()) for w in wins)
    bw = 6 * 8 - 1
    kspec = {
        # Schur block accumulation: 216 flop per (obs_h, obs_l) pair; compulsory bytes = the W and Y
        # tiles (2 x 18 doubles per optimised observation) read once + S written once
        2: ("hbm", opt_obs * 36 * 8.0 + W * (6 * F) * (bw + 1) * 8.0, "GB/s"),
        # linearisation: residual + 2x3 + 2x6 Jacobian per observation: reads pose/point/uv, writes 20 doubles
        3: ("hbm", n_obs * (20 * 8.0 + 16 + 8) + 0.0, "GB/s"),
        # banded Cholesky + 2 triangular solves: n*bw^2 + 4*n*bw flops
        4: ("fp64", W * ((6 * F) * bw * bw + 4.0 * (6 * F) * bw), "TFLOP/s"),
    }
    return dict(step=step, check=check, ba_iters=10.0 * W, matches=float(W * nq), pairs=pairs,
                it_flops=it_flops, plan_ms=plan_ms, cleanup=plan.close, kspec=kspec,
                config={"workload": "c4_local_mapping_step", "windows_per_gpu": W, "kf": F, "fixed_kf": 5,
                        "points": n_pts // W, "observations": n_obs // W, "lm_iterations": 10,
                        "new_kf_keypoints": nq, "match": f"{nq}x{nt} bf crossCheck"},
                cpu=lambda: cpu_baseline_c4(steps[0]))


def cpu_baseline_c4(st, budget_s=12.0):
    """Oracle (C restatement of the reference path, TEST INFRASTRUCTURE) timed on host cores:
    the same step on a bounded sample (1 window: match + unproject + 10 LM iterations)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    fp = synth.frame_params()
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    n, t_match, t_ba = 0, 0.0, 0.0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s or n == 0:
        a = time.perf_counter()
        O.bf_match(st["kf_desc"], st["mp_desc"])
        O.unproject_stereo(fp, st["kf_Tcw"], st["kf_x"], st["kf_y"], st["kf_depth"])
        b = time.perf_counter()
        O.ba_local([st["window"]], opt)
        c = time.perf_counter()
        t_match += b - a; t_ba += c - b; n += 1
    dt = time.perf_counter() - t0
    return {"value": 10.0 * n / dt, "unit": "BA iterations/s", "cores": 1, "kind": "port",
            "matches_per_sec": 2000.0 * n / dt, "stage_s": {"match+unproject": t_match / n, "ba_10_its": t_ba / n},
            "sample": f"{n} x C4 local-mapping step (1 window), oracle C restatement gcc -O2, 1 thread "
                      f"(Ceres default num_threads=1), {dt:.1f}s"}


def workload_shared(ctx, args, rank, D):
    """BASELINE C5 shared-window variant: ONE 50-KF window with 80,000 points
    (~600,000 observations) point-partitioned over the N ranks, 10 LM iterations per step with
    the three RCCL all-reduces per iteration; plus the new keyframe's 2,000 descriptors matched
    (crossCheck) against the window's 80,000 map-point descriptors with the query rows split over
    the ranks.  Strong scaling: total work is fixed as N grows."""
    from lorb_slam_amd import shard
    from lorb_slam_amd.runtime import Comm, unique_id
    world = D.world
    win = synth.ba_window(seed=11, n_kf=50, n_pts=args.shared_points, n_fixed=5, fixed_obs_per_kf=400)
    sh = shard.shard_window(win, rank, world)
    uid = unique_id() if rank == 0 else None
    uid = D.broadcast_bytes(uid)
    comm = Comm.rccl(ctx, world, rank, uid)
    t0 = time.perf_counter()
    plan = BAPlan(ctx, [sh], comm=comm)
    plan_ms = (time.perf_counter() - t0) * 1e3
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    rng = np.random.default_rng(12)
    nq, nt = 2000, args.shared_points
    mp_desc = synth.random_desc(rng, nt)
    kf_desc = synth.random_desc(rng, nq)
    a, b = nq * rank // world, nq * (rank + 1) // world
    dq, dt = ctx.to_device(kf_desc[a:b] if b > a else kf_desc[:1]), ctx.to_device(mp_desc)
    q_off = np.array([0, b - a], np.int32)
    q_base = np.array([a], np.int32)
    t_off = np.array([0, nt], np.int32)
    outs = [ctx.empty(max(b - a, 1), np.int32) for _ in range(3)]
    nm = ctx.empty(1, np.int32)
    L = lib()

    def step():
        ctx.check(L.lorb_bf_match_sharded_dev(ctx.handle, comm.handle, C.c_int32(1), dq.as_ptr(C.c_uint8),
                                              A.ptr(q_off, C.c_int32), A.ptr(q_base, C.c_int32), dt.as_ptr(C.c_uint8),
                                              A.ptr(t_off, C.c_int32), *[o.as_ptr(C.c_int32) for o in outs],
                                              nm.as_ptr(C.c_int32)), "lorb_bf_match_sharded_dev")
        plan.solve(opt)

    def check():
        _, _, summ = plan.read()
        return {"n_matches": int(nm.numpy()[0]), "ba_final_cost": summ[0]["final_cost"],
                "ba_iterations": summ[0]["iterations"]}

    def cleanup():
        plan.close()
        comm.close()

    n_obs = len(win["obs_point"])
    kp = np.bincount(sh["obs_point"][sh["obs_frame"] >= 0])
    pt_flops = float(np.sum(60 + 108 * kp + 108 * kp * (kp + 1)))
    pair_cnt = float(np.sum(kp * (kp + 1) // 2))
    opt_obs = int((sh["obs_frame"] >= 0).sum())
    bw = 6 * 8 - 1
    kspec = {
        2: ("hbm", opt_obs * 36 * 8.0 + (6 * 50) * (bw + 1) * 8.0, "GB/s"),
        3: ("hbm", len(sh["obs_point"]) * (20 * 8.0 + 16 + 8), "GB/s"),
        4: ("fp64", (6 * 50) * bw * bw + 4.0 * (6 * 50) * bw, "TFLOP/s"),
    }
    del pair_cnt, pt_flops
    # whole-job units: the shared window's iterations / matches are counted once (rank 0 only)
    return dict(step=step, check=check, ba_iters=10.0 if rank == 0 else 0.0, matches=float(nq) if rank == 0 else 0.0,
                pairs=float(b - a) * nt, it_flops=0.0, plan_ms=plan_ms, cleanup=cleanup, kspec=kspec,
                config={"workload": "c5_shared_window", "kf": 50, "fixed_kf": 5, "points": len(win["point_init"]),
                        "observations": n_obs, "lm_iterations": 10, "new_kf_keypoints": nq,
                        "match": f"{nq}x{nt} bf crossCheck, query rows sharded", "points_this_rank": len(sh["point_init"])},
                cpu=None, scaling="strong")


def workload_c2(ctx, args, rank):
    """BASELINE config 1: brute-force Hamming 2000x2000 random 256-bit + ratio test, batched
    over `pairs` independent frame pairs per GPU."""
    B = args.pairs
    qs, ts, ls = [], [], []
    for p in range(B):
        q, t, lev = synth.bf_problem(seed=1000 * rank + p, nq=2000, nt=2000, n_planted=1000, random_levels=True)
        qs.append(q); ts.append(t); ls.append(lev)
    q_off = np.arange(B + 1, dtype=np.int32) * 2000
    t_off = np.arange(B + 1, dtype=np.int32) * 2000
    dq, dt, dl = ctx.to_device(np.concatenate(qs)), ctx.to_device(np.concatenate(ts)), ctx.to_device(np.concatenate(ls))
    nq = B * 2000
    outs = [ctx.empty(nq, np.int32) for _ in range(5)]
    acc = ctx.empty(nq, np.uint8)
    L = lib()

    def step():
        ctx.check(L.lorb_bf_top2_dev(ctx.handle, C.c_int32(B), dq.as_ptr(C.c_uint8), A.ptr(q_off, C.c_int32),
                                     dt.as_ptr(C.c_uint8), A.ptr(t_off, C.c_int32), dl.as_ptr(C.c_int32),
                                     *[o.as_ptr(C.c_int32) for o in outs], acc.as_ptr(C.c_uint8)), "bf_top2_dev")

    def cpu():
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        threads = max(1, min(16, os.cpu_count() or 1))
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 10.0 or n == 0:
            O.bf_top2(qs[0], ts[0], ls[0], threads=threads)
            n += 1
        d = time.perf_counter() - t0
        return {"value": n * 2000 / d, "unit": "matches/s", "cores": threads, "kind": "port",
                "sample": f"{n} x (2000x2000 bf top-2 + ratio test), oracle C -O2, {threads} threads, {d:.1f}s"}

    return dict(step=step, check=lambda: {"accepted": int(acc.numpy().sum())}, ba_iters=0.0, matches=float(nq),
                pairs=float(nq) * 2000, it_flops=0.0, plan_ms=0.0, cleanup=lambda: None, kspec={},
                config={"workload": "c2_bf_top2_ratio", "pairs_per_gpu": B, "nq": 2000, "nt": 2000}, cpu=cpu)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes (FETCH_SIZE and
    WRITE_SIZE collected in separate runs, gfx950 FETCH_SIZE x2 correction; tools/pmc_traffic.py).
    PMC counters cannot be read live from inside the timed process, so this is the profiled
    value of the same command; null when no summary is committed."""
    try:
        with open(TRAFFIC) as f:
            tab = json.load(f)
    except (OSError, ValueError):
        return None
    ent = tab.get("kernels", {}).get(kernel)
    return None if ent is None else ent.get("hbm_bytes_per_launch")


def roofline_entry(kt, wl, steps):
    """Dominant kernel (largest total device time in the profile pass) vs its roofline."""
    best = max(kt.items(), key=lambda kv: kv[1][0]) if kt else None
    if not best or best[1][1] == 0:
        return None
    k, (ms, n) = best
    avg_s = ms / n * 1e-3
    per_step = n / steps
    if k in (0, 1):
        amount = wl["pairs"] * OPS_PER_PAIR / per_step
        bound, peak, unit = "valu_int32", INT32_VALU_PEAK, "Tops/s"
    else:
        kind, amount, unit = wl["kspec"][k]
        # FP64 kernels (the Cholesky's SYRK runs on v_mfma_f64_16x16x4f64) are priced against the
        # dense FP64 peak, which is the same for MFMA and VALU on MI355X
        bound, peak = ("hbm", HBM_PEAK) if kind == "hbm" else ("mfma", FP64_PEAK)
    achieved = amount / avg_s
    scale = 1e9 if unit == "GB/s" else 1e12
    name = K_NAMES.get(k, str(k))
    return {"bound": bound, "achieved": achieved / scale, "peak": peak / scale, "unit": unit,
            "frac": achieved / peak, "traffic": pmc_traffic(K_PROF.get(k, name)), "kernel": name,
            "algorithmic_per_launch": amount, "avg_kernel_us": avg_s * 1e6, "launches_per_step": per_step,
            "all_kernels_ms_per_step": {K_NAMES.get(kk, str(kk)): v[0] / steps for kk, v in kt.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=["c4", "c2", "shared"])
    ap.add_argument("--shared-points", type=int, default=80000)
    ap.add_argument("--windows", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    D = Dist()
    # one rank per GPU; with fewer GPUs than ranks (a rehearsal on a 1-GPU box) ranks share them
    ndev = device_count()
    ctx = Context(D.local_rank % ndev if ndev > 0 else D.local_rank)
    if args.workload == "shared":
        wl = workload_shared(ctx, args, D.rank, D)
    else:
        wl = (workload_c4 if args.workload == "c4" else workload_c2)(ctx, args, D.rank)
    for _ in range(args.warmup):
        wl["step"]()
    ctx.sync()
    D.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl["step"]()
    ctx.sync()
    t1 = time.perf_counter()
    D.barrier()
    elapsed = D.reduce(t1 - t0, "MAX")
    check = wl["check"]()
    # profile pass (same steps, per-kernel HIP events; BA runs eagerly instead of as a graph)
    L = lib()
    kernel_times(ctx, range(8))
    L.lorb_kernel_timing_enable(ctx.handle, 1)
    prof_steps = max(3, min(args.steps, 10))
    for _ in range(prof_steps):
        wl["step"]()
    ctx.sync()
    kt = {k: v for k, v in kernel_times(ctx, range(8)).items() if v[1] > 0}
    L.lorb_kernel_timing_enable(ctx.handle, 0)
    total_iters = D.reduce(wl["ba_iters"] * args.steps, "SUM")
    total_matches = D.reduce(wl["matches"] * args.steps, "SUM")
    cpu = wl["cpu"]() if (D.rank == 0 and not args.no_cpu_baseline and D.world == 1 and wl["cpu"]) else None
    if D.rank == 0:
        if args.workload in ("c4", "shared"):
            value, unit = total_iters / elapsed, "BA iterations/s"
        else:
            value, unit = total_matches / elapsed, "matches/s"
        rf = roofline_entry(kt, wl, prof_steps)
        out = {
            "metric": METRIC, "value": value, "unit": unit, "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": wl.get("scaling", "weak"), "vs_baseline": None, "dtype": "f64+u8", "data": "synthetic",
            "config": dict(wl["config"], parallelism=(f"point-partitioned window over {D.world} ranks (RCCL)"
                                                      if args.workload == "shared" else f"independent windows x{D.world}")),
            "matches_per_sec": total_matches / elapsed, "plan_build_ms": wl["plan_ms"],
            "roofline": rf, "cpu_baseline": cpu, "check": check,
        }
        print(json.dumps(out))
    wl["cleanup"]()
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
