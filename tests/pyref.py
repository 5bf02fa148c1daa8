"""Independent pure-Python restatement (small cases only) of the windowed matchers, used to pin
the C oracle.  float32 arithmetic is reproduced with numpy float32 scalars; reference
file:line cited per function."""
import math

import numpy as np

f32 = np.float32


def descriptor_distance(a, b):  # src/matcher.cpp:369-385
    return int(np.bitwise_count(np.bitwise_xor(a, b)).sum())


def build_grid(fp, kps):  # src/frame.cpp:87-115
    grid = {}
    for i in range(len(kps["x"])):
        vx = f32(f32(kps["x"][i]) - f32(fp["min_x"])) * f32(fp["grid_w_inv"])
        vy = f32(f32(kps["y"][i]) - f32(fp["min_y"])) * f32(fp["grid_h_inv"])
        px = int(math.floor(float(vx) + 0.5)) if vx >= 0 else -int(math.floor(-float(vx) + 0.5))
        py = int(math.floor(float(vy) + 0.5)) if vy >= 0 else -int(math.floor(-float(vy) + 0.5))
        if px < 0 or px >= 64 or py < 0 or py >= 48:
            continue
        grid.setdefault((px, py), []).append(i)
    return grid


def features_in_area(fp, kps, grid, x, y, r, minLevel=-1, maxLevel=-1):  # src/frame.cpp:370-423
    x, y, r = f32(x), f32(y), f32(r)
    out = []
    x0 = max(0, int(math.floor(float(f32(f32(x - f32(fp["min_x"])) - r) * f32(fp["grid_w_inv"])))))
    if x0 >= 64:
        return out
    x1 = min(63, int(math.ceil(float(f32(f32(x - f32(fp["min_x"])) + r) * f32(fp["grid_w_inv"])))))
    if x1 < 0:
        return out
    y0 = max(0, int(math.floor(float(f32(f32(y - f32(fp["min_y"])) - r) * f32(fp["grid_h_inv"])))))
    if y0 >= 48:
        return out
    y1 = min(47, int(math.ceil(float(f32(f32(y - f32(fp["min_y"])) + r) * f32(fp["grid_h_inv"])))))
    if y1 < 0:
        return out
    check = minLevel > 0 or maxLevel >= 0
    for ix in range(x0, x1 + 1):
        for iy in range(y0, y1 + 1):
            for j in grid.get((ix, iy), []):
                oc = int(kps["octave"][j])
                if check:
                    if oc < minLevel:
                        continue
                    if maxLevel >= 0 and oc > maxLevel:
                        continue
                if abs(f32(kps["x"][j]) - x) < r and abs(f32(kps["y"][j]) - y) < r:
                    out.append(j)
    return out


def search_by_projection_local(fp, kps, slot_state, pts, th):  # src/matcher.cpp:220-316
    n = len(kps["x"])
    state = np.array(slot_state if slot_state is not None else np.zeros(n), np.uint8).copy()
    assign = -np.ones(n, np.int64)
    grid = build_grid(fp, kps)
    nm = 0
    for m in range(len(pts["proj_x"])):
        if not pts["track_in_view"][m] or (pts.get("is_bad") is not None and pts["is_bad"][m]):
            continue
        lev = int(pts["pred_level"][m])
        r = f32(2.5) if float(f32(pts["view_cos"][m])) > 0.998 else f32(4.0)
        if f32(th) != f32(1.0):
            r = f32(r * f32(th))
        rs = f32(r * f32(fp["scale_factors"][lev]))
        idx = features_in_area(fp, kps, grid, pts["proj_x"][m], pts["proj_y"][m], rs, lev - 1, lev)
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for j in idx:
            if state[j] == 2:
                continue
            if kps["u_right"][j] > 0 and abs(f32(pts["proj_xr"][m]) - f32(kps["u_right"][j])) > rs:
                continue
            d = descriptor_distance(pts["desc"][m], kps["desc"][j])
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(kps["octave"][j]), j
            elif d < bd2:
                bl2, bd2 = int(kps["octave"][j]), d
        if bd <= 100:
            if bl == bl2 and bd > 0.8 * bd2:
                continue
            assign[bi] = m
            state[bi] = 2 if pts["locked"][m] else 1
            nm += 1
    return assign, nm
