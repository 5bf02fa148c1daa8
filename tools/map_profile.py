"""Diagnostics: phase breakdown of the chained LocalMapping step (lorb_map_step_dev).

    LORB_MAP_PROFILE=1 python tools/map_profile.py [--steps 20]

The library syncs the stream after each phase and prints the mean host wall time per phase when
the map is destroyed; this script also prints the unsynchronised ms/step of the same stream."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import synth  # noqa: E402
from lorb_slam_amd.runtime import Context, LocalMap  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    seq = synth.mapping_sequence(steps=args.steps + 2)
    ctx = Context(0)
    opt = A.LMOptions.default(max_num_iterations=args.iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)
    fp = A.make_frame_params(synth.frame_params())
    M = LocalMap(ctx, seq["init"])
    kfs = [(k["pose"], k["Tcw"], len(k["x"]), ctx.to_device(A.u8(k["desc"])), ctx.to_device(A.f32(k["x"])),
            ctx.to_device(A.f32(k["y"])), ctx.to_device(A.f32(k["depth"]))) for k in seq["steps"]]
    M.step_dev(fp, *kfs[0][:3], *kfs[0][3:], opt=opt)
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(1, args.steps + 1):
        M.step_dev(fp, *kfs[i][:3], *kfs[i][3:], opt=opt)
    ctx.sync()
    dt = (time.perf_counter() - t0) / args.steps
    print(f"ms/step {dt * 1e3:.3f}  ({args.iters} LM its)  counts {M.counts()}  plan {M.plan_info()}", flush=True)
    M.close()
    ctx.close()


if __name__ == "__main__":
    main()
