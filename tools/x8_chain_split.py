"""Diagnostics: the chained C4 map step (bench.py's c4x8 sub-record) on 8 windows, with the maps
dealt to K contexts (streams) and K host threads, each thread stepping its 8 / K maps one after the
other (argv[3] == "group": as one lorb_map_group per context -- one set of BA launches per step).
K = 8 is the sub-record's round-5 layout.  Prints ms per 8-window step (argv[1] = K), overlap on
unless argv[2] == "0"."""
import concurrent.futures
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from lorb_slam_amd import _abi as A  # noqa: E402
from lorb_slam_amd import synth  # noqa: E402
from lorb_slam_amd.runtime import Context, LocalMap, MapGroup  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ovl = not (len(sys.argv) > 2 and sys.argv[2] == "0")
grp = len(sys.argv) > 3 and sys.argv[3] == "group"
W = 8
steps, warm = 20, 3
seqs = [synth.mapping_sequence(seed=4 + 17 * i, steps=steps + warm + 4) for i in range(W)]
opt = A.LMOptions.default(max_num_iterations=10, function_tolerance=0.0, gradient_tolerance=0.0, parameter_tolerance=0.0)
ctx0 = Context(0)
ctxs = [ctx0] + [Context(0) for _ in range(K - 1)]
owner = [i * K // W for i in range(W)]  # map i -> context
maps = [LocalMap(ctxs[owner[i]], seqs[i]["init"]) for i in range(W)]
for m in maps:
    m.set_overlap(ovl)
fp = A.make_frame_params(synth.frame_params())
kfs = [[(k["pose"], k["Tcw"], len(k["x"]), ctxs[owner[i]].to_device(A.u8(k["desc"])),
         ctxs[owner[i]].to_device(A.f32(k["x"])), ctxs[owner[i]].to_device(A.f32(k["y"])),
         ctxs[owner[i]].to_device(A.f32(k["depth"]))) for k in s["steps"]] for i, s in enumerate(seqs)]
pool = concurrent.futures.ThreadPoolExecutor(max_workers=K)
pos = [0]
groups = [MapGroup([maps[j] for j in range(W) if owner[j] == k]) for k in range(K)] if grp else None


def run_ctx(k):
    i = pos[0]
    if grp:
        groups[k].step_dev(fp, [kfs[j][i] for j in range(W) if owner[j] == k], opt)
        return
    for j in range(W):
        if owner[j] == k:
            pose, Tcw, n, dd, dx, dy, dz = kfs[j][i]
            maps[j].step_dev(fp, pose, Tcw, n, dd, dx, dy, dz, opt)


def step():
    for f in [pool.submit(run_ctx, k) for k in range(K)]:
        f.result()
    pos[0] += 1


for _ in range(warm):
    step()
for c in ctxs:
    c.sync()
t0 = time.perf_counter()
for _ in range(steps):
    step()
for c in ctxs:
    c.sync()
ms = (time.perf_counter() - t0) / steps * 1e3
costs = [m.read()["summary"]["final_cost"] for m in maps[:2]]
print("K=%d contexts, overlap %d, group %d: %.3f ms per 8-window step -> %.0f LM it/s (w0 cost %.9e)%s" %
      (K, ovl, grp, ms, 80.0 / (ms / 1e3), costs[0], " " + str(groups[0].info()) if grp else ""), flush=True)
if grp:
    for g in groups:
        g.close()
for m in maps:
    m.close()
pool.shutdown()
