#!/usr/bin/env python3
"""bench.py -- LORB_SLAM matcher + local-BA hot path on MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|shared|rehearse]

Launch.  The driver starts N>1 ranks itself (`torch.distributed.run ... bench.py --gpus N`).  When
`--gpus N > 1` is given without WORLD_SIZE in the environment, this script starts the N ranks
itself (a `torch.distributed.run` child process, before anything here touches a GPU) and exits
with its code.  A rank refuses to run (exit 2) when WORLD_SIZE != --gpus or when fewer devices
than ranks are visible: ranks never share a GPU silently.  `n_gpus` in the JSON line is the rank
count of the RCCL communicator the ranks build (ncclCommCount), not an argument echo.

Default workload (c4, BASELINE config "full local_mapping step -- match + triangulate + BA on a
50-KF / 10k-point sliding window"): per GPU, `--windows` independent HBM-resident local maps
(default 1, i.e. C4 at N=1 and C5 -- one window per GPU -- at N=8), each fed the next keyframe of
a synthetic stream every step (lorb_map_step_dev, the chained LocalMapping step):
  1. brute-force Hamming + OpenCV crossCheck + minDist filter of the new keyframe's 2,000
     descriptors against the map's ~10,000 point descriptors (Matcher::SearchLocalPoints),
  2. stereo unprojection of the keyframe's keypoints (Frame::UnprojectStereo),
  3. matches become observations, unmatched keypoints with depth become new points, the window
     slides by one keyframe (points no window keyframe sees leave), the BA plan of the slid window
     is built on the device (one small readback),
  4. 10 Levenberg-Marquardt iterations of BA::LocalPoseOptimization on the window (50 optimised
     KFs + 5 fixed, ~10,000 points, ~75,000 observations), tolerances 0, float write-back.
`value` = LM iterations/s over all GPUs.  The same run also times the BASELINE C2 matcher
config (batched 2000x2000 top-2 + ratio test) and reports it as the `c2` sub-record, so both
halves of the metric ("ORB matches/sec + local-BA iterations/sec") come from one driver run.

Inputs are synthetic (lorb_slam_amd.synth, seeded per rank) and resident in HBM before the
timed region.  torch.distributed (gloo, CPU) provides the barrier, the max-over-ranks of the
timing and the RCCL unique id; the data-path collectives (shared workload) are RCCL.
"""
import argparse
import concurrent.futures
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CLOCK = 2.4e9
INT32_VALU_PEAK = 256 * 4 * 32 * CLOCK      # lane-ops/s: 256 CU x 4 SIMD32 (MI355X_MICROARCH)
FP64_PEAK = 78.6e12                          # FP64 vector/matrix dense, MI355X spec
HBM_PEAK = 8.0e12                            # HBM3E spec (MI355X_MICROARCH)
OPS_PER_PAIR = 16                            # 8 x v_xor_b32 + 8 x v_bcnt_u32_b32 per 256-bit pair
# the Cholesky id covers three kernels chosen by band shape; C3/C4/C5 windows
# (band 47, n >= 128) run the two-sided k_ba_chol_2s
# Point-major BA path (the only Schur path since round 6): timer 3 is k_ba_ls (linearisation + point
# elimination + per-group Schur partials), timer 2 k_ba_red (the partials' fixed-order sum into the band)
K_NAMES = {0: "k_bf_scan<top2>", 1: "k_bf_scan<top1>", 2: "k_ba_red", 3: "k_ba_ls", 4: "k_ba_chol_2s"}
# rocprofv3 short names (tools/pmc_traffic.py) of the same kernels, for the PMC traffic lookup
# (the plan-group launches of map groups first, then partial runs, then the one-plan kernels)
K_PROF = {0: "k_bf_scan", 1: "k_bf_scan", 2: ("k_ba_red_g", K_NAMES[2]), 3: ("k_ba_ls_g", "k_ba_ls_sup", K_NAMES[3]),
          4: ("k_ba_chol_2s_g", "k_ba_chol_2s")}


def ba_kspec(W, n_obs, n_pts, F, bw):
    """Algorithmic bytes per launch of the BA kernels of W windows (id -> (bound, amount, unit)).
    Point-major: k_ba_ls reads per observation its uv (16 B) and three structure indices (12 B), per
    point X (24 B), and writes per point the point-block inverse and rhs (72 B); k_ba_red writes the
    band once."""
    band = W * (6 * F) * (bw + 1) * 8.0
    return {2: ("hbm", band, "GB/s"),
            3: ("hbm", W * (n_obs * 28.0 + n_pts * 96.0), "GB/s"),
            4: ("fp64", W * ((6 * F) * bw * bw + 4.0 * (6 * F) * bw), "TFLOP/s")}
# committed PMC summaries, newest first; each is keyed by workload (tools/pmc_traffic.py)
TRAFFIC = [os.path.join(ROOT, "profiles", r, "traffic.json") for r in ("r06", "r05", "r04", "r03", "r02", "r01")]
METRIC = "ORB matches/sec + local-BA iterations/sec (50 KF, 10k pts) at 1/2/4/8 MI355X"


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """Start n ranks as a torch.distributed.run child (no GPU has been touched in this process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def refuse(msg):
    print(f"bench.py: refusing to run: {msg}", file=sys.stderr, flush=True)
    sys.exit(2)


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


def host_cpu():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return model, avail


def cpu_threads():
    """host threads for the nproc leg: the cores this process may use, capped at the GPU box's
    per-GPU CPU share -- OMP_NUM_THREADS is 16 there and the pool's rules allot one GPU's job 16 of
    the host's hardware threads (the other GPUs' jobs share the rest), so 16 is the fair host-side
    comparison for one MI355X; the cap is stated next to every nproc number"""
    _, avail = host_cpu()
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(avail, cap, 16))


def run_parallel(fn, threads, budget_s):
    """fn() repeatedly on `threads` Python threads (the oracle's C calls release the GIL) for
    about budget_s; returns (completed calls, elapsed s)."""
    import threading
    stop = time.perf_counter() + budget_s
    counts = [0] * threads

    def worker(i):
        while True:
            fn()
            counts[i] += 1
            if time.perf_counter() >= stop:
                break
    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return sum(counts), time.perf_counter() - t0


def kernel_times(ctx, ids):
    from lorb_slam_amd.runtime import lib
    L = lib()
    out = {}
    for k in ids:
        ms, n = C.c_double(0), C.c_int(0)
        L.lorb_kernel_timing_read(ctx.handle, k, C.byref(ms), C.byref(n))
        out[k] = (ms.value, n.value)
    return out


# ------------------------------------------------------------------------------------------
def workload_c4(ctx, args, rank):
    """The chained LocalMapping step on an HBM-resident map (lorb_map_step_dev), one map per window:
    each step takes the next keyframe of a synthetic stream (synth.mapping_sequence), matches it
    against the map, appends observations and new points, slides the window by one keyframe, builds
    the BA plan on the device and runs 10 LM iterations.  The plan build is inside the step."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    from lorb_slam_amd.runtime import Context, LocalMap, MapGroup
    W = args.windows
    n_kf_needed = args.warmup + args.steps + max(3, min(args.steps, 10)) + 2
    seqs = [synth.mapping_sequence(seed=4 + 1009 * rank + 17 * i, steps=n_kf_needed) for i in range(W)]
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    # Several windows: map groups of G = 2 maps (lorb_map_group: per step the maps' match, append,
    # slide and plan build, then ONE set of BA launches for both windows), one context (stream) and
    # one host thread per group, so W / G groups step concurrently (the first on the caller's
    # context).  Measured on 8 C4 windows (tools/x8_chain_split.py): 4 groups of 2 1.97 ms
    # per 8-window step, 2 of 4 2.20, 1 of 8 3.43, and the round-5 layout -- one map, stream and
    # thread per window -- 2.44 (overlap off) / 2.62 ms (overlap on): HIP deals the streams to 4
    # hardware queues, and one group's Cholesky (one CU per window) runs beside another group's
    # point-group kernels.  One window: the map alone with the overlap of consecutive steps.
    G = 2 if W > 1 else 1
    ctxs = [ctx] + [Context(ctx.device) for _ in range((W + G - 1) // G - 1)]
    owner = [i // G for i in range(W)]
    t0 = time.perf_counter()
    maps = [LocalMap(ctxs[owner[i]], s["init"]) for i, s in enumerate(seqs)]
    groups = [MapGroup([maps[i] for i in range(W) if owner[i] == k]) for k in range(len(ctxs))] if W > 1 else None
    create_ms = (time.perf_counter() - t0) * 1e3
    # the keyframes below are uploaded (synchronously) before any step: step t+1's match and append
    # may run under step t's solve (lorb_map_set_overlap's requirement; tests/test_gpu_map.py checks
    # the overlapped chain bit-for-bit against the serial one)
    if W == 1:
        maps[0].set_overlap(True)
    fp = A.make_frame_params(synth.frame_params())
    # the keyframe stream, resident in HBM before the timed region
    kfs = [[(k["pose"], k["Tcw"], len(k["x"]), c.to_device(A.u8(k["desc"])), c.to_device(A.f32(k["x"])),
             c.to_device(A.f32(k["y"])), c.to_device(A.f32(k["depth"]))) for k in s["steps"]]
           for c, s in zip([ctxs[o] for o in owner], seqs)]
    pos = [0]

    # one host thread per group (each group's step blocks on its plans' readbacks; ctypes releases
    # the GIL inside the call), so the groups' host phases overlap
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=len(groups)) if groups else None

    def step():
        i = pos[0]
        if i >= n_kf_needed:
            raise RuntimeError("bench keyframe stream exhausted")
        if pool is None:
            pose, Tcw, n, dd, dx, dy, dz = kfs[0][i]
            maps[0].step_dev(fp, pose, Tcw, n, dd, dx, dy, dz, opt)
        else:
            def one(k):
                groups[k].step_dev(fp, [kfs[j][i] for j in range(W) if owner[j] == k], opt)
            for f in [pool.submit(one, k) for k in range(len(groups))]:
                f.result()
        pos[0] = i + 1

    def check():
        out = {"keyframes_stepped": pos[0], "windows": []}
        for i, m in enumerate(maps):
            st = m.read()
            if i == 0:  # the window of the last step, for roofline_iteration
                out["_window"] = {"obs_point": st["obs_point"], "obs_frame": st["obs_frame"], "point_init": st["point"]}
            out["windows"].append({k: st[k] for k in ("t0", "points", "observations", "matches", "new_points")}
                                  | {"ba_final_cost": st["summary"]["final_cost"],
                                     "ba_iterations": st["summary"]["iterations"]})
        return out

    c = maps[0].counts()
    n_obs, n_pts = c["observations"], c["points"]
    F = maps[0].W
    nq = len(seqs[0]["steps"][0]["x"])
    bw = 6 * 8 - 1
    opt_obs = n_obs  # window observations; the fixed ones (~4%) are in n_obs too
    # per launch: the profile pass times the first context's launches, each over its group's G windows
    kspec = ba_kspec(G, opt_obs, n_pts, F, bw)

    def cleanup():
        for g in groups or []:
            g.close()
        for m in maps:
            m.close()
        for ks in kfs:
            for k in ks:
                for a in k[3:]:
                    a.free()
        for c in ctxs[1:]:
            c.close()
        if pool is not None:
            pool.shutdown()

    def sync():
        for c in ctxs:
            c.sync()

    return dict(step=step, check=check, sync=sync, maps=maps, ba_iters=10.0 * W, matches=float(W * nq), pairs=float(W) * nq * n_pts,
                plan_ms=0.0, create_ms=create_ms, cleanup=cleanup, kspec=kspec, traffic_key="c4_chain",
                config={"workload": "c4_local_mapping_step_chained", "windows_per_gpu": W, "kf": F,
                        **({"map_groups": f"{len(groups)} x {G} windows (lorb_map_group), one stream each"} if groups else {}),
                        "fixed_kf": maps[0].F, "points": n_pts, "observations": n_obs, "lm_iterations": 10,
                        "new_kf_keypoints": nq, "match": f"{nq}x~{n_pts} bf crossCheck",
                        "step": "match + unproject + append + slide/cull + device plan build + 10 LM its + write-back"},
                cpu=lambda: cpu_baseline_c4(seqs[0], args.cpu_budget))


def sub_c4x8(ctx, D, args):
    """A filled GPU: the C4 chained step on 8 independent HBM-resident windows per
    GPU, stepped together (each step issues one keyframe to every window; north_star shards
    independent windows).  The windows run as 4 map groups of 2 (lorb_map_group: one set of BA
    launches per group and step), one context (stream) and host thread per group,
    so the groups' steps run concurrently.  One window leaves most CUs idle during its Cholesky; this
    line shows what one MI355X sustains with 8 in flight.  It does not replace the headline (one
    window).  Its roofline comes from the profile pass, where per-kernel events make each group
    solve its plans one after another (the same kernels per window)."""
    import copy
    a = copy.copy(args)
    a.windows, a.steps, a.warmup = 8, max(10, min(args.steps, 20)), max(2, min(args.warmup, 3))
    wl = workload_c4(ctx, a, D.rank)
    elapsed = timed(ctx, D, wl, a.steps, a.warmup)
    chk = wl["check"]()
    rwin = chk.pop("_window", None)
    kt, pn = profile_pass(ctx, wl, a.steps)
    total = D.reduce(wl["ba_iters"] * a.steps, "SUM")
    ms = elapsed / a.steps * 1e3
    wl["traffic_key"] = "c4x8"
    out = {"workload": "c4_local_mapping_step_chained_x8", "config": wl["config"], "value": total / elapsed,
           "unit": "BA iterations/s", "steps": a.steps, "ms_per_step": ms,
           "roofline": roofline_entry(kt, wl, pn),
           # per window-iteration: the step's time / (10 iterations x 8 windows)
           "roofline_iteration": roofline_iteration(rwin, wl["config"]["kf"], ms / (10.0 * a.windows), "c4x8", 2)
           if rwin is not None else None,
           "check": {"windows": chk["windows"][:2], "keyframes_stepped": chk["keyframes_stepped"]}}
    wl["cleanup"]()
    out["one_plan"] = c4x8_one_plan(ctx, D, a.steps)
    return out


def c4x8_one_plan(ctx, D, steps):
    """The LM solve alone on 8 independent C4 windows in ONE plan (every point-group, block and
    Cholesky kernel launched once for all 8 windows; tests/test_gpu_ba.py
    test_local_ba_eight_c4_windows_independent checks it bit for bit against 8 one-window plans):
    10 LM iterations per solve, the plan built once outside the timed solves.  `four_plans_x2`: the
    same 8 windows as 4 plans of 2 on 4 contexts (streams), the 4 solves enqueued back to back --
    the layout of the c4x8 map groups."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    from lorb_slam_amd.runtime import BAPlan, Context
    wins = [synth.ba_window(seed=40 + i, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400) for i in range(8)]
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)

    def timed_solves(plans, ctxs):
        for _ in range(2):
            for p in plans:
                p.solve(opt)
        for c in ctxs:
            c.sync()
        D.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            for p in plans:
                p.solve(opt)
        for c in ctxs:
            c.sync()
        return D.reduce(time.perf_counter() - t0, "MAX")

    plan = BAPlan(ctx, wins)
    try:
        el = timed_solves([plan], [ctx])
        s = plan.read()[2]
    finally:
        plan.close()
    ctxs = [ctx] + [Context(ctx.device) for _ in range(3)]
    plans = [BAPlan(c, wins[2 * k:2 * k + 2]) for k, c in enumerate(ctxs)]
    try:
        el4 = timed_solves(plans, ctxs)
        s4 = plans[0].read()[2]
    finally:
        for p in plans:
            p.close()
        for c in ctxs[1:]:
            c.close()
    ms, ms4 = el / steps * 1e3, el4 / steps * 1e3
    return {"workload": "c4_local_ba_x8_one_plan", "value": D.reduce(80.0 * steps, "SUM") / el,
            "unit": "BA iterations/s", "solves": steps, "ms_per_solve": ms,
            "roofline_iteration": roofline_iteration(wins[0], 50, ms / 80.0, "c4x8"),
            "check": {"final_cost_w0": s[0]["final_cost"], "iterations_w0": s[0]["iterations"]},
            "four_plans_x2": {"value": D.reduce(80.0 * steps, "SUM") / el4, "unit": "BA iterations/s",
                              "ms_per_8_windows": ms4, "final_cost_w0": s4[0]["final_cost"],
                              "same_as_one_plan": s4[0]["final_cost"] == s[0]["final_cost"]}}


def sub_c4x8_run(ctx, D, args):
    """The c4x8 sub-record.  On one rank it runs in a child process of its own: measured after the
    single-window headline in the same process, the 8 windows' steps ran ≈ 25 % slower (3.4 vs
    2.6 ms per 8-window step, tools/c4x8_host.py --headline, also with the headline's map closed):
    the streams created before them change how HIP deals the windows' streams to its hardware
    queues (see workload_c4), and the sub-record should not depend on what ran before it.  The
    child touches the GPU only while this process waits for it."""
    if D.world > 1:
        return sub_c4x8(ctx, D, args)
    ctx.sync()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.abspath(__file__), "--c4x8-child", "--steps", str(args.steps), "--warmup", str(args.warmup)]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        raise RuntimeError(f"c4x8 child failed (rc={r.returncode})")
    out = json.loads(lines[-1])
    out["process"] = "child (fresh process)"
    return out


def cpu_baseline_c4(seq, budget_s):
    """Oracle (restatement of the reference path, TEST INFRASTRUCTURE) timed on host cores on a
    bounded sample of the same chained step (1 window: crossCheck match + unproject + append/slide +
    10 LM iterations, from the same starting map every call): at 1 thread (Ceres' default
    num_threads=1) and at the host's thread count (independent windows in flight)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_map import MapOracle
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    fp = synth.frame_params()
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    base = MapOracle(seq["init"]).state()
    kf = seq["steps"][0]
    intr = seq["init"]["intr"]

    def one():
        MapOracle.from_state(base, intr).step(fp, kf, opt)
    n1, d1 = run_parallel(one, 1, budget_s)
    nt = cpu_threads()
    nn, dn = run_parallel(one, nt, budget_s) if nt > 1 else (n1, d1)
    model, avail = host_cpu()
    nq = len(kf["x"])
    return {"value": 10.0 * n1 / d1, "unit": "BA iterations/s", "cores": 1, "kind": "port",
            "matches_per_sec": nq * n1 / d1, "steps_per_sec": n1 / d1,
            "sample": f"{n1} x C4 chained local-mapping step (1 window: {nq}x{len(base['point'])} crossCheck + "
                      f"unproject + append/slide + 10 LM its), oracle C restatement gcc -O3 + numpy bookkeeping, "
                      f"1 thread (Ceres default num_threads=1), {d1:.1f}s",
            "nproc": {"value": 10.0 * nn / dn, "cores": nt, "matches_per_sec": nq * nn / dn,
                      "sample": f"{nn} steps on {nt} threads (independent windows; {nt} = the box's per-GPU CPU share), {dn:.1f}s"},
            "host_cpu": model, "host_cpus_available": avail}


C1_PAIRS = 32  # distinct frame pairs the C1 timings cycle through (every call sees new inputs)


def c1_inputs(n=C1_PAIRS):
    """n distinct C1 frame pairs (synth.two_frames seeds 1..n: 2 x 500 kps, 200 shared map points)
    with their a2 train sets and a12 problems (200 residuals each)"""
    from lorb_slam_amd import synth
    out = []
    for s in range(1, n + 1):
        pr = synth.two_frames(seed=s, n_kps=500, n_shared=200)
        last = pr["last"]
        out.append(dict(pr=pr, tdesc=np.ascontiguousarray(last["mp_desc"][last["has_mp"] > 0]),
                        pb=synth.pose_only_batch(seed=s, n_frames=1, n_res=200)))
    return out


def c1_calls(x, L, handle=None):
    """The three C1 calls on input set x as zero-argument closures over PRE-MARSHALLED ctypes
    arguments (the caller's arrays, structs and output buffers built once, outside the timing), so
    that a timing covers the C-ABI call itself: a2 BF crossCheck, a4 SearchByProjection(th 15),
    a12 ProjectPoseOptimization.  handle=None: the oracle library (or_*), else liblorb on that ctx."""
    from lorb_slam_amd import _abi as A
    keep = A.KeepAlive()
    pr, tdesc, pb = x["pr"], x["tdesc"], x["pb"]
    cur, last = pr["cur_kps"], pr["last"]
    q = keep.keep(A.u8(cur["desc"]).reshape(-1, 32))
    t = keep.keep(A.u8(tdesc).reshape(-1, 32))
    nq = len(q)
    o3 = [keep.keep(np.zeros(max(nq, 1), np.int32)) for _ in range(3)]
    nm1 = keep.keep(np.zeros(1, np.int32))
    qo = keep.keep(np.array([0, nq], np.int32))
    to = keep.keep(np.array([0, len(t)], np.int32))
    fps = A.make_frame_params(pr["fp"])
    k = A.make_keypoints(cur, keep)
    lf = A.make_last_frame(last, keep)
    T = keep.keep(A.f32(pr["cur_Tcw"]).reshape(16))
    ss = keep.keep(A.u8(pr["slot_state"])) if pr["slot_state"] is not None else None
    assign = keep.keep(np.empty(max(1, k.n), np.int32))
    nm = C.c_int32(0)
    s = A.make_pose_batch(pb, keep)
    opt = A.LMOptions.default()
    pose = keep.keep(np.zeros((s.n_frames, 6)))
    Tp = keep.keep(np.zeros((s.n_frames, 4, 4), np.float32))
    summ = (A.BASummary * max(1, s.n_frames))()
    ptr = A.ptr
    if handle is None:
        calls = {
            "a2_bf_match": lambda: L.or_bf_match(ptr(q, C.c_uint8), C.c_int(nq), ptr(t, C.c_uint8), C.c_int(len(t)),
                                                 ptr(o3[0], C.c_int32), ptr(o3[1], C.c_int32), ptr(o3[2], C.c_int32)),
            "a4_search_by_projection_th15": lambda: L.or_search_by_projection_frame(
                C.byref(fps), ptr(T, C.c_float), C.byref(k), ptr(ss, C.c_uint8), C.byref(lf), C.c_float(15.0),
                ptr(assign, C.c_int32), C.byref(nm)),
            "a12_pose_only_200": lambda: L.or_ba_pose_only(C.byref(s), C.byref(opt), ptr(pose, C.c_double),
                                                           ptr(Tp, C.c_float), summ)}
    else:
        def chk(rc):
            if rc != 0:
                raise RuntimeError(f"C1 call failed: {rc}")
        calls = {
            "a2_bf_match": lambda: chk(L.lorb_bf_match(handle, C.c_int32(1), ptr(q, C.c_uint8), ptr(qo, C.c_int32),
                                                       ptr(t, C.c_uint8), ptr(to, C.c_int32), ptr(o3[0], C.c_int32),
                                                       ptr(o3[1], C.c_int32), ptr(o3[2], C.c_int32), ptr(nm1, C.c_int32))),
            "a4_search_by_projection_th15": lambda: chk(L.lorb_search_by_projection_frame(
                handle, C.byref(fps), ptr(T, C.c_float), C.byref(k), ptr(ss, C.c_uint8), C.byref(lf), C.c_float(15.0),
                ptr(assign, C.c_int32), C.byref(nm))),
            "a12_pose_only_200": lambda: chk(L.lorb_ba_pose_only(handle, C.byref(s), C.byref(opt), ptr(pose, C.c_double),
                                                                 ptr(Tp, C.c_float), summ))}
    return calls, (keep, fps, k, lf, nm, s, opt, summ)


def sub_c1(ctx, D, args):
    """BASELINE C1 on the GPU through the host C-ABI (the calls a per-frame caller issues): the a2 BF
    crossCheck match, SearchByProjection(curr, last, 15) (a4) and ProjectPoseOptimization of 200
    matched points (a12), host arrays in and out, synchronous.  Every call takes the next of 32
    distinct frame pairs (new inputs each time: nothing is resident from an earlier call); median
    over 3 passes of the 32.  Latency-bound: a few thousand items per call."""
    from lorb_slam_amd.runtime import lib
    xs = c1_inputs()
    prepared = [c1_calls(x, lib(), ctx.handle) for x in xs]
    per = {}
    for name in prepared[0][0]:
        prepared[0][0][name]()
        ts = []
        for _ in range(3):
            for calls, _ in prepared:
                t0 = time.perf_counter()
                calls[name]()
                ts.append(time.perf_counter() - t0)
        per[name] = D.reduce(float(np.median(ts)), "MAX") * 1e3
    total = sum(per.values())
    return {"workload": "c1_two_frames_500kps", "value": 1e3 / total, "unit": "C1 sequences/s (a2 + a4 + a12)",
            "ms_per_sequence": total, "stage_ms_median": per, "distinct_inputs": len(xs),
            "call": "host C-ABI (lorb_bf_match, lorb_search_by_projection_frame, lorb_ba_pose_only), synchronous, "
                    "timed around the ctypes call with the arguments marshalled beforehand; the inputs packed into "
                    "one pinned staging buffer that one kernel pulls into HBM, the results stored by the last "
                    "kernel straight into pinned memory"}


def cpu_baseline_c1(budget_s):
    """BASELINE C1 (the reference's CPU-runnable case): two synthetic frames of 500 ORB
    keypoints, 200 shared map points -- the BF crossCheck match of the current frame against the last
    frame's map points (a2), SearchByProjection(curr, last, 15) (a4) and ProjectPoseOptimization of
    the 200 matched points (a12) -- on the oracle (C restatement, gcc -O3 -ffp-contract=off), 1
    thread, median of >= 30 runs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    xs = c1_inputs()
    prepared = [c1_calls(x, O.lib()) for x in xs]
    per = {}
    t_end = time.perf_counter() + budget_s
    for name in prepared[0][0]:
        ts = []
        while len(ts) < 3 * len(xs) or (time.perf_counter() < t_end and len(ts) < 2000):
            calls = prepared[len(ts) % len(xs)][0]
            t0 = time.perf_counter()
            calls[name]()
            ts.append(time.perf_counter() - t0)
        per[name] = float(np.median(ts)) * 1e3
    total = sum(per.values())
    return {"value": 1e3 / total, "unit": "C1 sequences/s (a2 + a4 + a12)", "cores": 1, "kind": "port",
            "ms_per_sequence": total, "stage_ms_median": per,
            "sample": f"{len(xs)} distinct pairs of 2 frames x 500 kps, 200 shared MPs (synth.two_frames seeds 1..{len(xs)}): "
                      "a2 + a4 th=15 + a12, oracle C gcc -O3 -ffp-contract=off, timed around the ctypes call with "
                      "the arguments marshalled beforehand (as the GPU leg), 1 thread, median of >= 96 runs per stage"}


def workload_c3(ctx, args, rank):
    """BASELINE config 2: local BA on 20 keyframes / 4,000 points / 30,000 window
    observations (+2 fixed keyframes, 800 observations), exactly 10 LM iterations (tolerances 0).
    A step = the device-built plan of the resident window (lorb_ba_plan_update_dev: the reference
    rebuilds its Ceres problem every call) + the 10-iteration solve from the initial values."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    from lorb_slam_amd.runtime import BAPlanDev
    w = synth.ba_window(seed=3 + 1009 * rank, n_kf=20, n_pts=4000, n_fixed=2, fixed_obs_per_kf=400)
    # observation slots grouped by point (stable), the order the reference's BA adds its residual
    # blocks in (map point by map point, src/bundle_adjust.cpp:240-280) and the HBM map keeps: the
    # device plan build takes its sorted path
    order = np.argsort(np.asarray(w["obs_point"]), kind="stable")
    w = dict(w, **{k: np.asarray(w[k])[order] for k in ("obs_point", "obs_frame", "obs_uv")})
    arrays = BAPlanDev.upload(ctx, w)
    t0 = time.perf_counter()
    plan = BAPlanDev(ctx, arrays, 20, 2, w["intr"])
    ctx.sync()
    plan_ms = (time.perf_counter() - t0) * 1e3
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)

    def step():
        plan.update()
        plan.solve(opt)

    def check():
        _, _, summ = plan.read()
        return {"ba_final_cost": summ[0]["final_cost"], "ba_iterations": summ[0]["iterations"]}

    def cleanup():
        plan.close()
        for x in arrays.values():
            x.free()

    n_obs, n_pts, F = len(w["obs_point"]), len(w["point_init"]), 20
    bw = 6 * 8 - 1
    kspec = ba_kspec(1, n_obs, n_pts, F, bw)  # the C4 figures of workload_c4 for this window

    def cpu():
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        budget = max(2.0, args.cpu_budget / 2)
        n1, d1 = run_parallel(lambda: O.ba_local([w], opt), 1, budget)
        nt = cpu_threads()
        nn, dn = run_parallel(lambda: O.ba_local([w], opt), nt, budget) if nt > 1 else (n1, d1)
        model, avail = host_cpu()
        return {"value": 10.0 * n1 / d1, "unit": "BA iterations/s", "cores": 1, "kind": "port",
                "sample": f"{n1} x C3 solve (10 LM its, Schur + dense LLT), oracle C restatement gcc -O3, "
                          f"1 thread (Ceres default num_threads=1), {d1:.1f}s",
                "nproc": {"value": 10.0 * nn / dn, "cores": nt,
                          "sample": f"{nn} solves on {nt} threads (independent windows; {nt} = the box's per-GPU CPU share), {dn:.1f}s"},
                "host_cpu": model, "host_cpus_available": avail}

    return dict(step=step, check=check, ba_iters=10.0, matches=0.0, pairs=0.0, plan_ms=plan_ms, cleanup=cleanup,
                kspec=kspec, traffic_key="c3", window=w, n_poses=F,
                config={"workload": "c3_local_ba", "kf": F, "fixed_kf": 2, "points": n_pts, "observations": n_obs,
                        "window_observations": int((np.asarray(w["obs_frame"]) >= 0).sum()), "lm_iterations": 10,
                        "step": "device-built plan of the resident window + 10 LM its from the initial values"},
                cpu=cpu)


def sub_c3(ctx, D, args):
    """BASELINE C3 (20 KF / 4k points / 30k observations, 10 LM its) inside the default run."""
    wl = workload_c3(ctx, args, D.rank)
    steps = max(10, min(args.steps, 100))
    elapsed = timed(ctx, D, wl, steps, max(2, args.warmup))
    kt, pn = profile_pass(ctx, wl, steps)
    total = D.reduce(wl["ba_iters"] * steps, "SUM")
    chk = wl["check"]()
    cpu = wl["cpu"]() if (D.rank == 0 and not args.no_cpu_baseline and D.world == 1) else None
    ms = elapsed / steps * 1e3
    out = {"workload": wl["config"]["workload"], "config": wl["config"], "value": total / elapsed,
           "unit": "BA iterations/s", "steps": steps, "ms_per_step": ms, "plan_create_ms": wl["plan_ms"],
           "roofline": roofline_entry(kt, wl, pn),
           "roofline_iteration": roofline_iteration(wl["window"], wl["n_poses"], ms / 10.0, "c3"),
           "cpu_baseline": cpu, "check": chk}
    wl["cleanup"]()
    return out


def workload_shared(ctx, args, rank, D, comm):
    """BASELINE C5 shared-window variant: ONE 50-KF window with 80,000 points
    (~600,000 observations) point-partitioned over the N ranks (each rank's points with all of their
    observations, resident in HBM).  A step is: the new keyframe's 2,000 descriptors matched
    (crossCheck) against the window's 80,000 map-point descriptors with the query rows split over
    the ranks, the device-built sharded BA plan rebuilt from the resident shard (collective: one
    all-reduce of the camera structure), and 10 LM iterations with three RCCL all-reduces each.
    Strong scaling: total work is fixed as N grows."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import shard, synth
    from lorb_slam_amd.runtime import BAPlanDev, lib
    world = comm.size()[0] if comm is not None else 1
    win = synth.ba_window(seed=11, n_kf=50, n_pts=args.shared_points, n_fixed=5, fixed_obs_per_kf=400)
    sh = shard.shard_window(win, rank, world)
    arrays = BAPlanDev.upload(ctx, sh)
    t0 = time.perf_counter()
    plan = BAPlanDev(ctx, arrays, 50, 5, win["intr"], comm=comm)
    ctx.sync()
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
        plan.update()
        plan.solve(opt)

    def check():
        _, _, summ = plan.read()
        return {"n_matches": int(nm.numpy()[0]), "ba_final_cost": summ[0]["final_cost"],
                "ba_iterations": summ[0]["iterations"]}

    def cleanup():
        plan.close()
        for x in (dq, dt, nm, *outs, *arrays.values()):
            x.free()

    n_obs = len(win["obs_point"])
    opt_obs = int((sh["obs_frame"] >= 0).sum())
    bw = 6 * 8 - 1
    kspec = ba_kspec(1, len(sh["obs_point"]), len(sh["point_init"]), 50, bw)  # this rank's shard
    # whole-job units: the shared window's iterations / matches are counted once (rank 0 only)
    return dict(step=step, check=check, ba_iters=10.0 if rank == 0 else 0.0, matches=float(nq) if rank == 0 else 0.0,
                pairs=float(b - a) * nt, plan_ms=plan_ms, cleanup=cleanup, kspec=kspec,
                traffic_key=f"shared_w{world}", n_ranks=world, window=win, n_poses=50,
                config={"workload": "c5_shared_window", "kf": 50, "fixed_kf": 5, "points": len(win["point_init"]),
                        "observations": n_obs, "lm_iterations": 10, "new_kf_keypoints": nq,
                        "match": f"{nq}x{nt} bf crossCheck, query rows sharded", "points_this_rank": len(sh["point_init"]),
                        "step": "sharded match + device-built sharded plan (collective) + 10 LM its (3 RCCL all-reduces each)"},
                cpu=None, scaling="strong")


def workload_c2(ctx, args, rank):
    """BASELINE config 1: brute-force Hamming 2000x2000 random 256-bit + ratio test, batched
    over `pairs` independent frame pairs per GPU (each pair is a full 2000x2000 problem with its
    own seeded descriptors: every problem of the batch is distinct)."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    from lorb_slam_amd.runtime import lib
    B = args.pairs
    U = B
    gen = [synth.bf_problem(seed=1000 * rank + p, nq=2000, nt=2000, n_planted=1000, random_levels=True) for p in range(U)]
    qs = [gen[p % U][0] for p in range(B)]
    ts = [gen[p % U][1] for p in range(B)]
    ls = [gen[p % U][2] for p in range(B)]
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
        budget = max(2.0, args.cpu_budget / 2)
        n1, d1 = run_parallel(lambda: O.bf_top2(qs[0], ts[0], ls[0]), 1, budget)
        nt = cpu_threads()
        nn, dn = run_parallel(lambda: O.bf_top2(qs[0], ts[0], ls[0]), nt, budget) if nt > 1 else (n1, d1)
        model, avail = host_cpu()
        return {"value": n1 * 2000 / d1, "unit": "matches/s", "cores": 1, "kind": "port",
                "sample": f"{n1} x (2000x2000 bf top-2 + ratio test), oracle C -O3, 1 thread, {d1:.1f}s",
                "nproc": {"value": nn * 2000 / dn, "cores": nt,
                          "sample": f"{nn} problems on {nt} threads ({nt} = the box's per-GPU CPU share), {dn:.1f}s"},
                "host_cpu": model, "host_cpus_available": avail}

    def cleanup():
        for a in (dq, dt, dl, acc, *outs):
            a.free()

    return dict(step=step, check=lambda: {"accepted": int(acc.numpy().sum())}, ba_iters=0.0, matches=float(nq),
                pairs=float(nq) * 2000, plan_ms=0.0, cleanup=cleanup, kspec={}, traffic_key="c2",
                config={"workload": "c2_bf_top2_ratio", "pairs_per_gpu": B, "unique_pairs": U, "nq": 2000, "nt": 2000},
                cpu=cpu)


class _NullCtx:
    def sync(self):
        pass

    def close(self):
        pass


def workload_rehearse(ctx, args, rank):
    """Launcher / gloo rehearsal without a GPU: a fixed CPU busy-step per rank.  Exercises the
    rank spawn, barrier, max-over-ranks timing and the single JSON line; its value measures
    nothing about the hot path (the line says so)."""
    a = np.random.default_rng(rank).standard_normal((128, 128))

    def step():
        for _ in range(4):
            a @ a
    return dict(step=step, check=lambda: {}, ba_iters=1.0, matches=0.0, pairs=0.0, plan_ms=0.0,
                cleanup=lambda: None, kspec={}, traffic_key=None,
                config={"workload": "rehearsal_cpu_no_gpu"}, cpu=None)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` in `workload` from the committed rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE collected in separate runs; the gfx950 FETCH_SIZE correction per kernel
    from tools/micro/fetch_cal.hip's calibration, x2 for streaming kernels and x1 for record gathers;
    tools/pmc_traffic.py).  PMC counters cannot be read live from inside the timed process, so
    this is the profiled value of the same command; null when no summary for this workload
    and kernel is committed."""
    for path in TRAFFIC:
        try:
            with open(path) as f:
                tab = json.load(f)
        except (OSError, ValueError):
            continue
        wls = tab.get("workloads") or {"c4": tab}  # r01 files hold the c4 workload only
        for name in (kernel if isinstance(kernel, tuple) else (kernel,)):
            ent = wls.get(workload, {}).get("kernels", {}).get(name)
            if ent is not None and ent.get("hbm_bytes_per_launch") is not None:
                return {"hbm_bytes_per_launch": ent["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT),
                        "kernel": name}
    return None


def roofline_entry(kt, wl, steps):
    """Dominant kernel (largest total device time in the profile pass) vs its roofline."""
    # kernels with an algorithmic figure only (the all-reduce timer, K 7, is not a kernel)
    cand = {k: v for k, v in kt.items() if k in (0, 1) or k in wl.get("kspec", {})}
    best = max(cand.items(), key=lambda kv: kv[1][0]) if cand else None
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
    tr = pmc_traffic(wl["traffic_key"], K_PROF.get(k, name)) if wl.get("traffic_key") else None
    return {"bound": bound, "achieved": achieved / scale, "peak": peak / scale, "unit": unit,
            "frac": achieved / peak, "traffic": tr["hbm_bytes_per_launch"] if tr else None,
            "traffic_source": tr["source"] if tr else None, "kernel": tr["kernel"] if tr else name,
            "algorithmic_per_launch": amount, "avg_kernel_us": avg_s * 1e6, "launches_per_step": per_step,
            "all_kernels_ms_per_step": {K_NAMES.get(kk, str(kk)): v[0] / steps for kk, v in kt.items()}}


def pmc_bytes_per_iteration(workload, group=1):
    """HBM bytes per LM iteration of the BA kernels (k_ba_*: every launch of a solve, k_ba_init's
    amortised) from this round's committed PMC summary, with the per-kernel breakdown; None when the
    workload has no summary.  Iterations = k_ba_lm_end launches (one per LM iteration), plus `group`
    window-iterations per k_ba_lm_end_g launch (a plan group's)."""
    for path in TRAFFIC:
        try:
            with open(path) as f:
                tab = json.load(f)
        except (OSError, ValueError):
            continue
        ks = (tab.get("workloads") or {}).get(workload, {}).get("kernels", {})
        its = ks.get("k_ba_lm_end", {}).get("calls", 0) + group * ks.get("k_ba_lm_end_g", {}).get("calls", 0)
        if not its:
            continue
        per = {k: e["calls"] * e["hbm_bytes_per_launch"] / its for k, e in ks.items()
               if k.startswith("k_ba_") and e.get("hbm_bytes_per_launch") is not None and e.get("calls")}
        return {"bytes": sum(per.values()), "per_kernel": per, "source": os.path.relpath(path, ROOT)}
    return None


def roofline_iteration(win, n_poses, ms_per_iteration, traffic_key, group=1):
    """SURVEY §8(d)'s whole-iteration roofline of one LM iteration on a window:
       F_it = sum_obs 380 + sum_pts (60 + 108 k_p + 108 k_p (k_p + 1)) + (6F)^3 / 3 + 4 (6F)^2 + sum_obs 40
       B_it = 24 N_obs + 48 N_pts + 16 (6F)^2
    (k_p = window observations of point p, F = optimised poses; the (6F)^3/3 term is the dense LLT
    that §8(d) prices, not the banded one this build runs), against the measured time per iteration
    (the whole step / 10: conservative, it includes the match and the plan build), with the PMC
    bytes per iteration beside B_it."""
    obs_point = np.asarray(win["obs_point"])
    opt = np.asarray(win["obs_frame"]) >= 0
    n_obs = len(obs_point)
    n_pts = len(win["point_init"])
    kp = np.bincount(obs_point[opt], minlength=n_pts).astype(np.float64)
    n6 = 6.0 * n_poses
    f_it = 420.0 * n_obs + float(np.sum(60.0 + 108.0 * kp + 108.0 * kp * (kp + 1.0))) + n6 ** 3 / 3.0 + 4.0 * n6 ** 2
    b_it = 24.0 * n_obs + 48.0 * n_pts + 16.0 * n6 ** 2
    t = ms_per_iteration * 1e-3
    pmc = pmc_bytes_per_iteration(traffic_key, group)
    return {"flop_per_iteration": f_it, "bytes_per_iteration": b_it, "ms_per_iteration": ms_per_iteration,
            "achieved_tflops": f_it / t / 1e12, "peak_tflops": FP64_PEAK / 1e12, "frac_fp64": f_it / t / FP64_PEAK,
            "achieved_gbs": b_it / t / 1e9, "peak_gbs": HBM_PEAK / 1e9, "frac_hbm": b_it / t / HBM_PEAK,
            "pmc_bytes_per_iteration": pmc["bytes"] if pmc else None,
            "pmc_over_algorithmic": pmc["bytes"] / b_it if pmc else None,
            "pmc_per_kernel": pmc["per_kernel"] if pmc else None, "traffic_source": pmc["source"] if pmc else None,
            "definition": "SURVEY 8(d) F_it / B_it per LM iteration; time = step / 10"}


def timed(ctx, D, wl, steps, warmup):
    """W untimed steps, then exactly K steps bracketed by barrier + device sync; max over ranks."""
    sync = wl.get("sync", ctx.sync)  # every stream the workload runs on
    for _ in range(warmup):
        wl["step"]()
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl["step"]()
    sync()
    t1 = time.perf_counter()
    D.barrier()
    return D.reduce(t1 - t0, "MAX")


def profile_pass(ctx, wl, steps):
    """the same steps again with per-kernel HIP events on the context stream (BA runs eagerly
    instead of as a graph); returns {kernel id: (total ms, launches)} and the step count"""
    from lorb_slam_amd.runtime import lib
    L = lib()
    kernel_times(ctx, range(8))
    L.lorb_kernel_timing_enable(ctx.handle, 1)
    n = max(3, min(steps, 10))
    for _ in range(n):
        wl["step"]()
    wl.get("sync", ctx.sync)()
    kt = {k: v for k, v in kernel_times(ctx, range(8)).items() if v[1] > 0}
    L.lorb_kernel_timing_enable(ctx.handle, 0)
    return kt, n


def sub_c2(ctx, D, args):
    """BASELINE C2 (2000x2000 top-2 + ratio test, `--pairs` pairs per GPU) inside the default run."""
    wl = workload_c2(ctx, args, D.rank)
    steps = max(5, args.steps)
    elapsed = timed(ctx, D, wl, steps, max(2, args.warmup))
    kt, pn = profile_pass(ctx, wl, steps)
    total = D.reduce(wl["matches"] * steps, "SUM")
    chk = wl["check"]()
    cpu = wl["cpu"]() if (D.rank == 0 and not args.no_cpu_baseline and D.world == 1) else None
    wl["cleanup"]()
    return {"workload": wl["config"]["workload"], "config": wl["config"], "value": total / elapsed,
            "unit": "matches/s", "pairs_per_sec": total * 2000 / elapsed, "steps": steps,
            "ms_per_step": elapsed / steps * 1e3, "roofline": roofline_entry(kt, wl, pn),
            "cpu_baseline": cpu, "check": chk}


def workload_shared_rehearse(ctx, args, rank, D, comm):
    """CPU rehearsal of the shared sub-record (no GPU): the same three exchanges per LM iteration,
    sized as the C5 window's (camera blocks + costs, the S band + rhs, the step sums), all-reduced
    over gloo, so the launcher, the sub-record's keys and its max-over-ranks timing are exercised.
    It measures nothing about the hot path."""
    import torch
    bufs = [torch.zeros(n, dtype=torch.float64) for n in (50 * 27 + 2, 32 * 10 + 300 * 48, 3)]

    def step():
        for _ in range(10):
            for b in bufs:
                D.dist.all_reduce(b) if D.dist else None

    def profile(steps):
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ms = (time.perf_counter() - t0) * 1e3
        return {7: (ms, 3 * 10 * steps)}, steps
    return dict(step=step, check=lambda: {}, ba_iters=10.0 if rank == 0 else 0.0, matches=0.0, pairs=0.0,
                plan_ms=0.0, cleanup=lambda: None, kspec={}, traffic_key=None, profile=profile, n_ranks=D.world,
                config={"workload": "rehearsal_shared_exchanges_cpu"}, cpu=None, scaling="strong")


def sub_shared(ctx, D, args, comm):
    """BASELINE C5 shared-window variant inside the default run: the point-partitioned
    window over the N ranks of this job, strong scaling, with the per-iteration time of the three
    RCCL all-reduces from the profile pass (HIP events around the collectives on the ctx stream)."""
    rehearse = args.workload == "rehearse"
    wl = (workload_shared_rehearse if rehearse else workload_shared)(ctx, args, D.rank, D, comm)
    steps = max(5, min(args.steps, 20))
    elapsed = timed(ctx, D, wl, steps, max(2, args.warmup))
    kt, pn = wl["profile"](steps) if rehearse else profile_pass(ctx, wl, steps)
    chk = wl["check"]()
    total = D.reduce(wl["ba_iters"] * steps, "SUM")
    ar = kt.pop(7, (0.0, 0))
    its = 10.0 * pn
    ar_ms = D.reduce(ar[0] / its if its else 0.0, "MAX")
    wl["cleanup"]()
    ms = elapsed / steps * 1e3
    # SURVEY 8(d)'s per-iteration figures of the WHOLE window (all ranks' points); the PMC bytes are
    # this rank's (at one rank: the whole window)
    rit = (roofline_iteration(wl["window"], wl["n_poses"], ms / 10.0, wl["traffic_key"])
           if wl.get("window") is not None else None)
    return {"workload": wl["config"]["workload"], "n_ranks": wl["n_ranks"], "scaling": "strong",
            "value": total / elapsed, "unit": "BA iterations/s", "steps": steps, "ms_per_step": ms,
            "plan_create_ms": wl["plan_ms"], "allreduce_ms_per_iteration": ar_ms,
            "allreduce_launches_per_iteration": (ar[1] / its) if its else 0.0,
            "roofline": roofline_entry(kt, wl, pn), "roofline_iteration": rit, "config": wl["config"], "check": chk}


def sub_dropin(ctx, D, args):
    """The drop-in BA::LocalPoseOptimization call (include/lorb/adapters.hpp -> lorb_ba_solver_solve):
    a C4 window (50 KF + 5 fixed, 10,000 points, ~77 k observations) in the reference's camera order
    ([curr] + covisible by ascending weight, src/bundle_adjust.cpp:210-220), handed over as HOST arrays
    every call, 10 LM iterations, double results back on the host.  Each call = pack + one H2D copy +
    device plan build + LM graph + one D2H copy, synchronous, timed end to end on the host clock."""
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd import synth
    from lorb_slam_amd.runtime import BASolver
    w0 = synth.ba_window(seed=4 + 1009 * D.rank, n_kf=50, n_pts=10000, n_fixed=5, fixed_obs_per_kf=400)
    w, _ = synth.reference_window_order(w0)
    opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    s = BASolver(ctx)
    prep = s.prepare(w)
    t0 = time.perf_counter()
    s.solve_prepared(prep, opt)  # first call: plan creation + graph capture
    first_ms = (time.perf_counter() - t0) * 1e3
    for _ in range(max(2, args.warmup)):
        s.solve_prepared(prep, opt)
    steps = max(10, args.steps)
    D.barrier()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        s.solve_prepared(prep, opt)
        ts.append(time.perf_counter() - t0)
    D.barrier()
    _, _, summ = s.solve_prepared(prep, opt)
    info = s.info()
    s.close()
    mean = D.reduce(sum(ts) / steps, "MAX")
    med = D.reduce(float(np.median(ts)), "MAX")
    return {"workload": "dropin_local_ba_c4", "unit": "ms per call", "ms_per_call": mean * 1e3,
            "ms_per_call_median": med * 1e3, "first_call_ms": first_ms, "calls": steps,
            "lm_iterations_per_sec": 10.0 / mean,
            "config": {"kf": 50, "fixed_kf": 5, "points": len(w["point_init"]), "observations": len(w["obs_point"]),
                       "camera_order": "reference ([curr] + covisible by ascending weight)", "lm_iterations": 10,
                       "call": "lorb_ba_solver_solve: host arrays in, double results out (the adapter's C-ABI call)"},
            "solver": info, "final_cost": summ["final_cost"], "iterations": summ["iterations"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c4", choices=["c4", "c3", "c2", "shared", "rehearse"])
    ap.add_argument("--shared-points", type=int, default=80000)
    ap.add_argument("--windows", type=int, default=1)
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU-baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 sub-record of the default run")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in LocalPoseOptimization sub-record")
    ap.add_argument("--no-shared", action="store_true", help="skip the shared-window (RCCL) sub-record")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 local-BA sub-record")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 per-frame tracking sub-record")
    ap.add_argument("--no-c4x8", action="store_true", help="skip the 8-windows-per-GPU C4 sub-record")
    ap.add_argument("--c4x8-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        refuse(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    rehearse = args.workload == "rehearse"

    if rehearse:
        ctx = _NullCtx()
    else:
        from lorb_slam_amd.runtime import Context, device_count
        ndev = device_count()
        if ndev < world:
            refuse(f"{world} ranks but only {ndev} visible GPU(s); ranks never share a GPU")
    D = Dist()
    if args.c4x8_child:  # bench.py's own child for the c4x8 sub-record (sub_c4x8_run)
        from lorb_slam_amd.runtime import Context
        c = Context(0)
        print(json.dumps(sub_c4x8(c, D, args)), flush=True)
        c.close()
        return
    comm = None
    n_gpus = D.world

    def rccl_comm():
        from lorb_slam_amd.runtime import Comm, unique_id
        uid = D.broadcast_bytes(unique_id() if D.rank == 0 else None)
        return Comm.rccl(ctx, D.world, D.rank, uid)
    if not rehearse:
        ctx = Context(D.local_rank)
        if args.workload == "shared":  # the data path's collectives
            comm = rccl_comm()
            n_gpus = comm.size()[0]
    if args.workload == "shared":
        wl = workload_shared(ctx, args, D.rank, D, comm)
    else:
        wl = {"c4": workload_c4, "c3": workload_c3, "c2": workload_c2,
              "rehearse": workload_rehearse}[args.workload](ctx, args, D.rank)

    elapsed = timed(ctx, D, wl, args.steps, args.warmup)
    check = wl["check"]()
    rwin = check.pop("_window", None) if isinstance(check, dict) else None
    if rwin is None and wl.get("window") is not None:
        rwin = wl["window"]
    kt, pn = ({}, 1) if rehearse else profile_pass(ctx, wl, args.steps)
    total_iters = D.reduce(wl["ba_iters"] * args.steps, "SUM")
    total_matches = D.reduce(wl["matches"] * args.steps, "SUM")
    cpu = wl["cpu"]() if (D.rank == 0 and not args.no_cpu_baseline and D.world == 1 and wl["cpu"]) else None
    if cpu is not None and args.workload == "c4":
        cpu["c1"] = cpu_baseline_c1(max(2.0, args.cpu_budget / 2))
    c2 = sub_c2(ctx, D, args) if (args.workload == "c4" and not args.no_c2) else None
    dropin = sub_dropin(ctx, D, args) if (args.workload == "c4" and not args.no_dropin) else None
    c1 = sub_c1(ctx, D, args) if (args.workload == "c4" and not args.no_c1) else None
    c3 = sub_c3(ctx, D, args) if (args.workload == "c4" and not args.no_c3) else None
    c4x8 = sub_c4x8_run(ctx, D, args) if (args.workload == "c4" and args.windows == 1 and not args.no_c4x8) else None
    shared = None
    if args.workload in ("c4", "rehearse") and not args.no_shared:
        # the shared-window sub-record's communicator is created here, after the headline (which has
        # no collective: independent windows per rank), so that a communicator failure costs the
        # sub-record, not the headline line
        try:
            if not rehearse and comm is None:
                comm = rccl_comm()
            shared = sub_shared(ctx, D, args, comm)
        except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
            shared = {"error": f"{type(e).__name__}: {e}"}
    if D.rank == 0:
        if args.workload in ("c4", "c3", "shared"):
            value, unit = total_iters / elapsed, "BA iterations/s"
        elif args.workload == "c2":
            value, unit = total_matches / elapsed, "matches/s"
        else:
            value, unit = total_iters / elapsed, "rehearsal steps/s"
        par = (f"point-partitioned window over {D.world} ranks (RCCL)" if args.workload == "shared"
               else f"independent windows x{D.world}")
        out = {
            "metric": METRIC, "value": value, "unit": unit, "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": wl.get("scaling", "weak"), "vs_baseline": None, "dtype": "f64+u8",
            "data": "synthetic (lorb_slam_amd.synth, seeded per rank)",
            "config": dict(wl["config"], parallelism=par),
            "matches_per_sec": total_matches / elapsed, "plan_build_ms": wl["plan_ms"],
            "map_create_ms": wl.get("create_ms"),
            "roofline": roofline_entry(kt, wl, pn),
            "roofline_iteration": (roofline_iteration(rwin, wl.get("n_poses", wl["config"].get("kf", 50)),
                                                      elapsed / args.steps * 1e3 / max(wl["ba_iters"], 1.0),
                                                      wl["traffic_key"])
                                   if rwin is not None and wl["ba_iters"] > 0 else None),
            "cpu_baseline": cpu, "c2": c2, "c3": c3, "c4x8": c4x8, "dropin_local_ba": dropin, "shared": shared, "c1": c1,
            "check": check,
        }
        if rehearse:
            out["rehearsal"] = "no GPU: launcher + gloo path only; value is not a hot-path measurement"
        print(json.dumps(out), flush=True)
    wl["cleanup"]()
    if comm is not None:
        comm.close()
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
