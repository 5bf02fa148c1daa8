"""Independent pure-Python restatement (small cases only) of the windowed matchers, used to pin
the C oracle.  float32 arithmetic is reproduced with numpy float32 scalars; reference
file:line cited per function."""
import ctypes
import ctypes.util
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


def compute_stereo_matches(fp, left, right, pyr_l, pyr_r):  # src/frame.cpp:125-333
    """Pure-Python ComputeStereoMatches with the same defined behaviour at the edges as oracle/stereo.c
    (clipped bands, out-of-image windows => no depth, empty => no rejection).  Windows via numpy."""
    nL = len(left["x"])
    ur = np.full(nL, -1.0, np.float32); dp = np.full(nL, -1.0, np.float32)
    sf = [f32(s) for s in fp["scale_factors"]]
    nRows = pyr_l[0].shape[0]
    rows = [[] for _ in range(nRows)]
    for iR in range(len(right["x"])):  # :147-161
        kpY = f32(right["y"][iR]); r = f32(2.0) * sf[int(right["octave"][iR])]
        for yi in range(max(int(math.floor(f32(kpY - r))), 0), min(int(math.ceil(f32(kpY + r))), nRows - 1) + 1):
            rows[yi].append(iR)
    maxD = f32(fp["bf"]) / f32(fp["b"])
    pairs = []
    for iL in range(nL):  # :176-315
        lv = int(left["octave"][iL]); vL = f32(left["y"][iL]); uL = f32(left["x"][iL])
        if not (0 <= vL < nRows):
            continue
        cand = rows[int(vL)]
        if not cand:
            continue
        minU = f32(uL - maxD); maxU = uL
        if maxU < 0:
            continue
        best, bi = 100, 0
        for iR in cand:
            o = int(right["octave"][iR])
            if o < lv - 1 or o > lv + 1:
                continue
            uR = f32(right["x"][iR])
            if minU <= uR <= maxU:
                d = descriptor_distance(left["desc"][iL], right["desc"][iR])
                if d < best:
                    best, bi = d, iR
        if best >= 75:
            continue
        inv = f32(1.0) / sf[lv]
        su = int(np.round(f32(uL * inv))); sv = int(np.round(f32(vL * inv)))
        sr = int(np.round(f32(f32(right["x"][bi]) * inv)))
        IL, IR = pyr_l[lv].astype(np.int64), pyr_r[lv].astype(np.int64)
        h, w = IL.shape
        if sv - 5 < 0 or sv + 6 > h or su - 5 < 0 or su + 6 > w:
            continue
        if sr < 0 or sr + 11 >= pyr_r[lv].shape[1] or sr - 10 < 0:
            continue
        a = IL[sv - 5:sv + 6, su - 5:su + 6]; a = a - a[5, 5]
        dists = []
        for inc in range(-5, 6):
            b = IR[sv - 5:sv + 6, sr + inc - 5:sr + inc + 6]; b = b - b[5, 5]
            dists.append(int(np.abs(a - b).sum()))
        binc = int(np.argmin(dists)) - 5
        if binc in (-5, 5):
            continue
        d1, d2, d3 = f32(dists[binc + 4]), f32(dists[binc + 5]), f32(dists[binc + 6])
        with np.errstate(all="ignore"):
            delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if delta < -1 or delta > 1 or np.isnan(delta):
            if not np.isnan(delta):
                continue
        bu = f32(sf[lv] * f32(f32(f32(sr) + f32(binc)) + delta))
        disp = f32(uL - bu)
        if disp >= 0 and disp < maxD:
            if disp <= 0:
                disp = f32(0.01); bu = f32(float(uL) - 0.01)
            dp[iL] = f32(f32(fp["bf"]) / disp); ur[iL] = bu
            pairs.append((dists[binc + 5], iL))
    if pairs:  # :319-332
        pairs.sort()
        th = f32(f32(f32(1.5) * f32(1.4)) * f32(pairs[len(pairs) // 2][0]))
        for d, i in reversed(pairs):
            if f32(d) < th:
                break
            ur[i] = -1; dp[i] = -1
    return ur, dp, len(pairs)


def orb_blur(img):  # GaussianBlur 7x7 sigma 2 REFLECT_101, OpenCV 3.1 8U fixed point (via scipy)
    from scipy.ndimage import correlate1d
    cf = np.array([np.float32(math.exp(-0.125 * (i - 3) ** 2)) for i in range(7)], np.float32)
    s = 1.0 / float(np.sum(cf.astype(np.float64)))
    cf = np.array([np.float32(float(c) * s) for c in cf], np.float32)
    k = np.rint(cf * np.float32(256)).astype(np.int64)
    r = correlate1d(img.astype(np.int64), k, axis=1, mode="mirror")
    c = correlate1d(r, k, axis=0, mode="mirror")
    return np.clip((c + (1 << 15)) >> 16, 0, 255).astype(np.uint8)


def fast_atan2(y, x):  # cv::fastAtan2 (OpenCV 3.1) in float32
    k = f32(180 / math.pi)
    p1, p3 = f32(f32(0.9997878412794807) * k), f32(f32(-0.3258083974640975) * k)
    p5, p7 = f32(f32(0.1555786518463281) * k), f32(f32(-0.04432655554792128) * k)
    x, y = f32(x), f32(y)
    ax, ay = abs(x), abs(y)
    eps = f32(np.finfo(np.float64).eps)
    if ax >= ay:
        c = f32(ay / f32(ax + eps)); c2 = f32(c * c)
        a = f32(f32(f32(f32(f32(f32(f32(p7 * c2) + p5) * c2) + p3) * c2) + p1) * c)
    else:
        c = f32(ax / f32(ay + eps)); c2 = f32(c * c)
        a = f32(f32(90) - f32(f32(f32(f32(f32(f32(f32(p7 * c2) + p5) * c2) + p3) * c2) + p1) * c))
    if x < 0:
        a = f32(f32(180) - a)
    if y < 0:
        a = f32(f32(360) - a)
    return a


_LIBM = ctypes.CDLL(ctypes.util.find_library("m"))
_LIBM.cosf.restype = _LIBM.sinf.restype = ctypes.c_float
_LIBM.cosf.argtypes = _LIBM.sinf.argtypes = [ctypes.c_float]


def _cosf(v):
    return f32(_LIBM.cosf(float(f32(v))))


def _sinf(v):
    return f32(_LIBM.sinf(float(f32(v))))


def orb_describe(pyr, x, y, level, pattern):  # src/ORBextractor.cpp:79-150, 469-493, 1131-1132
    umax = np.zeros(16, np.int64)
    for v in range(0, 12):
        umax[v] = int(np.rint(math.sqrt(225 - v * v)))
    v0 = 0
    for v in range(15, 10, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    blurred = [orb_blur(p) for p in pyr]
    pat = np.asarray(pattern, np.int64).reshape(512, 2)
    ang = np.zeros(len(x), np.float32)
    desc = np.zeros((len(x), 32), np.uint8)
    for i in range(len(x)):
        img = pyr[level[i]].astype(np.int64)
        cx, cy = int(np.rint(f32(x[i]))), int(np.rint(f32(y[i])))
        m10 = m01 = 0
        for v in range(-15, 16):
            d = umax[abs(v)]
            row = img[cy + v, cx - d:cx + d + 1]
            u = np.arange(-d, d + 1)
            m10 += int((u * row).sum()); m01 += v * int(row.sum())
        ang[i] = fast_atan2(f32(m01), f32(m10))
        angle = f32(ang[i] * f32(math.pi / 180.0))
        a, b = _cosf(angle), _sinf(angle)  # std::cos(float) under `using namespace std` = libm cosf
        bl = blurred[level[i]]
        bits = []
        for p in range(512):
            px, py = f32(pat[p, 0]), f32(pat[p, 1])
            r = int(np.rint(f32(f32(px * b) + f32(py * a))))
            c = int(np.rint(f32(f32(px * a) - f32(py * b))))
            bits.append(int(bl[cy + r, cx + c]))
        t = np.array(bits).reshape(256, 2)
        bv = (t[:, 0] < t[:, 1]).astype(np.uint8).reshape(32, 8)
        desc[i] = (bv << np.arange(8, dtype=np.uint8)).sum(1).astype(np.uint8)
    return ang, desc


_OFF16 = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast(img, th):
    """cv::FAST 9-16 with non-maximum suppression, restated independently with numpy: a pixel is a
    corner if 9 contiguous circle pixels are all > v+th or all < v-th; its score is the largest t
    for which that still holds over some 9-arc (the max over arcs of the min |difference|) minus 1
    at the threshold floor -- computed here straight from that definition."""
    img = img.astype(np.int64)
    h, w = img.shape
    ring = np.stack([img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in _OFF16], 0)  # (16, h-6, w-6)
    v = img[3:h - 3, 3:w - 3]
    d = v[None] - ring                                    # center minus circle pixel
    ext = np.concatenate([d, d[:9]], 0)                   # 25 entries
    arcs_min = np.stack([ext[k:k + 9].min(0) for k in range(16)], 0)   # darker circle (d > 0)
    arcs_max = np.stack([ext[k:k + 9].max(0) for k in range(16)], 0)   # brighter circle (d < 0)
    dark = (arcs_min > th).any(0)
    bright = (arcs_max < -th).any(0)
    corner = dark | bright
    # cornerScore: a0 = max(th, max over 10-long windows' ...); restated as in the C restatement's
    # definition by brute force over the same arcs (k even starts, arcs [k..k+8] and [k+1..k+9])
    a0 = np.full(v.shape, th, np.int64)
    b0 = None
    for k in range(0, 16, 2):
        a = ext[k + 1:k + 9].min(0)
        a0 = np.maximum(a0, np.minimum(a, ext[k]))
        a0 = np.maximum(a0, np.minimum(a, ext[k + 9]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = ext[k + 1:k + 9].max(0)
        b0 = np.minimum(b0, np.maximum(b, ext[k]))
        b0 = np.minimum(b0, np.maximum(b, ext[k + 9]))
    score = np.where(corner, (-b0 - 1) & 0xFF, 0)
    S = np.zeros((h, w), np.int64)
    S[3:h - 3, 3:w - 3] = score
    C = np.zeros((h, w), bool)
    C[3:h - 3, 3:w - 3] = corner
    keep = C.copy()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dy or dx:
                keep &= S > np.roll(np.roll(S, -dy, 0), -dx, 1)
    ys, xs = np.nonzero(keep)  # row-major = FAST's emission order
    return xs.astype(np.float32), ys.astype(np.float32), S[ys, xs].astype(np.float32)


def resize_linear(img, h, w):  # OpenCV 3.1 8U INTER_LINEAR (imgwarp.cpp), numpy restatement
    sh, sw = img.shape

    def tabs(ss, ds, clamp):
        scale = 1.0 / (ds / ss)
        ofs, a0, a1, xmax = [], [], [], ds
        for d in range(ds):
            f = f32((d + 0.5) * scale - 0.5)
            s = int(np.floor(f))
            f = f32(f - f32(s))
            if clamp:
                if s < 0:
                    f, s = f32(0), 0
                if s + 1 >= ss:
                    xmax = min(xmax, d)
                    if s >= ss - 1:
                        f, s = f32(0), ss - 1
            ofs.append(s)
            a0.append(int(np.clip(np.rint(f32(f32(1) - f) * f32(2048)), -32768, 32767)))
            a1.append(int(np.clip(np.rint(f * f32(2048)), -32768, 32767)))
        return np.array(ofs), np.array(a0, np.int64), np.array(a1, np.int64), xmax

    xo, xa0, xa1, xmax = tabs(sw, w, True)
    yo, yb0, yb1, _ = tabs(sh, h, False)
    src = img.astype(np.int64)
    xs = 0
    while xs <= w - 16:
        xs += 16
    while xs < w - 4:
        xs += 4
    out = np.zeros((h, w), np.uint8)
    cols = np.arange(w)
    for dy in range(h):
        rows = []
        for k in (0, 1):
            sy = min(max(yo[dy] + k, 0), sh - 1)
            S = src[sy]
            nxt = S[np.minimum(xo + 1, sw - 1)]
            rows.append(np.where(cols < xmax, S[xo] * xa0 + nxt * xa1, S[xo] * 2048))
        b0, b1 = yb0[dy], yb1[dy]
        x0 = np.clip(rows[0] >> 4, -32768, 32767)
        y0 = np.clip(rows[1] >> 4, -32768, 32767)
        simd = np.clip(np.clip((x0 * b0 >> 16) + (y0 * b1 >> 16), -32768, 32767) + 2, -32768, 32767) >> 2
        scal = (rows[0] * b0 + rows[1] * b1 + (1 << 21)) >> 22
        out[dy] = np.clip(np.where(cols < xs, simd, scal), 0, 255).astype(np.uint8)
    return out


def orb_cells(rows, cols):
    """ComputeKeyPointsOctTree's cell grid (src/ORBextractor.cpp:803-847): list of
    (iniX, iniY, w, h) per cell, row-major, w = h = 0 for skipped cells."""
    W = f32(30)
    minb = 16
    maxbx, maxby = cols - 16, rows - 16
    width, height = f32(maxbx - minb), f32(maxby - minb)
    ncols, nrows = int(width / W), int(height / W)
    wcell, hcell = int(math.ceil(f32(width / f32(ncols)))), int(math.ceil(f32(height / f32(nrows))))
    cells = []
    for i in range(nrows):
        iy = minb + i * hcell
        my = min(iy + hcell + 6, maxby)
        for j in range(ncols):
            ix = minb + j * wcell
            mx = min(ix + wcell + 6, maxbx)
            if iy >= maxby - 3 or ix >= maxbx - 6:
                cells.append((ix, iy, 0, 0))
            else:
                cells.append((ix, iy, mx - ix, my - iy))
    return cells


def distribute_octree(kx, ky, resp, minX, maxX, minY, maxY, N):
    """DistributeOctTree (src/ORBextractor.cpp:554-797) restated with a Python list standing in for
    std::list<ExtractorNode> (push_front = insert at 0).  Nodes are [x0, y0, x1, y1, keys, creation];
    equal-size nodes sort by creation order (the pointer-order model of oracle/fast.c)."""
    kx = np.asarray(kx, np.float32); ky = np.asarray(ky, np.float32); resp = np.asarray(resp, np.float32)
    created = [0]

    def node(x0, y0, x1, y1):
        created[0] += 1
        return [x0, y0, x1, y1, [], created[0]]

    def divide(p):
        hx = int(math.ceil(f32(f32(p[2] - p[0]) / f32(2))))
        hy = int(math.ceil(f32(f32(p[3] - p[1]) / f32(2))))
        mx, my = p[0] + hx, p[1] + hy
        c = [node(p[0], p[1], mx, my), node(mx, p[1], p[2], my), node(p[0], my, mx, p[3]), node(mx, my, p[2], p[3])]
        for k in p[4]:
            q = (0 if ky[k] < my else 2) if kx[k] < mx else (1 if ky[k] < my else 3)
            c[q][4].append(k)
        return c

    n_ini = int(math.floor(float(f32(maxX - minX) / f32(maxY - minY)) + 0.5))  # std::round(float)
    hX = f32(f32(maxX - minX) / f32(n_ini))
    nodes = [node(int(f32(hX * f32(i))), 0, int(f32(hX * f32(i + 1))), maxY - minY) for i in range(n_ini)]
    for k in range(len(kx)):
        nodes[int(f32(kx[k] / hX))][4].append(k)
    nodes = [n for n in nodes if n[4]]
    finish = False
    pairs = []
    while not finish:
        prev = len(nodes)
        pairs = []
        n_expand = 0
        i = 0
        while i < len(nodes):
            n = nodes[i]
            if len(n[4]) == 1:
                i += 1
                continue
            kids = [c for c in divide(n) if c[4]]
            for c in kids:                      # push_front n1..n4
                nodes.insert(0, c)
                if len(c[4]) > 1:
                    n_expand += 1
                    pairs.append(c)
            i += len(kids)
            del nodes[i]                        # erase the divided node
        if len(nodes) >= N or len(nodes) == prev:
            finish = True
        elif len(nodes) + 3 * n_expand > N:
            while not finish:
                prev = len(nodes)
                todo = sorted(pairs, key=lambda c: (len(c[4]), c[5]))
                pairs = []
                for p in reversed(todo):
                    for c in [c for c in divide(p) if c[4]]:
                        nodes.insert(0, c)
                        if len(c[4]) > 1:
                            pairs.append(c)
                    nodes.remove(p)
                    if len(nodes) >= N:
                        break
                if len(nodes) >= N or len(nodes) == prev:
                    finish = True
    out = []
    for n in nodes:
        best = n[4][0]
        for k in n[4][1:]:
            if resp[k] > resp[best]:
                best = k
        out.append(best)
    return np.array(out, np.int32)
