"""Independent pure-Python restatement of the reference hot path, for small known-answer cases.

TEST INFRASTRUCTURE ONLY. Written directly from GuassianSplatting/tiled_shaders.metal and
tiled_rasterizer.mm (file:line cited per function) with numpy float32 / float16 scalars, in the
same evaluation order as the MSL text; no code is shared with oracle/gs_oracle.c. It is slow
(per-pixel Python loops) and used only on scenes of a few dozen splats to cross-check the C oracle,
which is then the checker for the GPU path.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
f16 = np.float16
SH_C0 = f32(0.28209479177387814)  # tiled_shaders.metal:83


def fmaf(a, b, c):
    # a*b is exact in float64 for float32 inputs; one rounding of the sum to float64, then to
    # float32 (double rounding is harmless for the moderate magnitudes used here)
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def expf(x) -> np.float32:
    """The pinned exp of the reference semantics (see oracle/gs_oracle.c gso_expf)."""
    x = f32(x)
    if x != x:
        return x
    if x > f32(88.0):
        return f32(np.inf)
    if x < f32(-87.0):
        return f32(0.0)
    k = f32(np.rint(f32(x * f32(1.44269502))))
    r = fmaf(k, f32(-0.693145751953125), x)
    r = fmaf(k, f32(-1.42860677e-06), r)
    p = f32(1.98756915e-4)
    for c in (1.39819995e-3, 8.33345191e-3, 4.16657959e-2, 1.66666655e-1, 5.00000012e-1):
        p = fmaf(p, r, f32(c))
    r2 = f32(r * r)
    y = f32(fmaf(p, r2, r) + f32(1.0))
    return f32(y * f32(2.0 ** int(k)))


def h(x) -> np.float16:
    return f16(f32(x))


def mat3_mul(A, B):
    """Metal float3x3 (A*B)[j][i] = sum_k A[k][i] * B[j][k], summed in k order."""
    C = [[f32(0)] * 3 for _ in range(3)]
    for j in range(3):
        for i in range(3):
            s = f32(A[0][i] * B[j][0])
            s = f32(s + f32(A[1][i] * B[j][1]))
            s = f32(s + f32(A[2][i] * B[j][2]))
            C[j][i] = s
    return C


def transpose(A):
    return [[A[r][c] for r in range(3)] for c in range(3)]


def quat_to_mat(w, x, y, z):
    """tiled_shaders.metal:91-99 (columns as listed)."""
    one, two = f32(1), f32(2)
    return [
        [f32(one - two * f32(f32(y * y) + f32(z * z))), f32(two * f32(f32(x * y) + f32(w * z))),
         f32(two * f32(f32(x * z) - f32(w * y)))],
        [f32(two * f32(f32(x * y) - f32(w * z))), f32(one - two * f32(f32(x * x) + f32(z * z))),
         f32(two * f32(f32(y * z) + f32(w * x)))],
        [f32(two * f32(f32(x * z) + f32(w * y))), f32(two * f32(f32(y * z) - f32(w * x))),
         f32(one - two * f32(f32(x * x) + f32(y * y)))],
    ]


def mat4_vec(M, v):
    out = []
    for r in range(4):
        s = f32(M[0 * 4 + r] * v[0])
        for c in (1, 2, 3):
            s = f32(s + f32(M[c * 4 + r] * v[c]))
        out.append(s)
    return out


def clamp(x, lo, hi):
    return f32(min(max(f32(x), f32(lo)), f32(hi)))


def project(g, u):
    """projectGaussians (tiled_shaders.metal:102-304) for one Gaussian -> dict of the 88-B fields."""
    p = dict(screen=(f32(0), f32(0)), conic=(f32(0),) * 3, depth=f32(0), opacity=f32(0),
             color=(f32(0),) * 3, radius=f32(0), tmin=(0xFFFFFFFF, 0xFFFFFFFF), tmax=(0, 0),
             vxy=(f32(0), f32(0)), cov=(f32(0),) * 3)
    pos = [f32(v) for v in g[0:3]]
    sc = [f32(v) for v in g[4:7]]
    if any(math.isnan(v) for v in pos + sc) or any(abs(v) > f32(1e6) for v in pos):
        return p
    world = pos + [f32(1)]
    view = mat4_vec(u[0:16], world)
    clip = mat4_vec(u[32:48], world)
    if clip[3] <= f32(0.1) or view[2] <= f32(0.1):
        return p
    ndc = [f32(clip[0] / clip[3]), f32(clip[1] / clip[3])]
    if abs(ndc[0]) > f32(1.2) or abs(ndc[1]) > f32(1.2):
        return p
    W, H = f32(u[48]), f32(u[49])
    sx = f32(f32(f32(ndc[0] * f32(0.5)) + f32(0.5)) * W)
    sy = f32(f32(f32(ndc[1] * f32(0.5)) + f32(0.5)) * H)
    p["screen"] = (sx, sy)
    p["depth"] = view[2]
    p["vxy"] = (view[0], view[1])
    s = [expf(clamp(v, -5.0, 5.0)) for v in sc]
    mx, mn = max(max(s[0], s[1]), s[2]), min(min(s[0], s[1]), s[2])
    if mx > f32(f32(20) * mn):
        f = f32(f32(f32(20) * mn) / mx)
        s = [f32(v * f) for v in s]
    q = [f32(v) for v in g[8:12]]
    qd = f32(q[0] * q[0])
    for k in (1, 2, 3):
        qd = f32(qd + f32(q[k] * q[k]))
    ql = f32(math.sqrt(float(qd)))  # sqrt of a float32 is exact in double, then rounded once
    q = [f32(v / ql) for v in q] if ql > f32(0.001) else [f32(1), f32(0), f32(0), f32(0)]
    R = quat_to_mat(*q)
    S = [[s[0], f32(0), f32(0)], [f32(0), s[1], f32(0)], [f32(0), f32(0), s[2]]]
    M = mat3_mul(R, S)
    Sigma = mat3_mul(M, transpose(M))
    z = view[2]
    fx, fy = f32(u[50]), f32(u[51])
    limx, limy = f32(f32(f32(1.3) * fx) / z), f32(f32(f32(1.3) * fy) / z)
    txtz = clamp(f32(view[0] / z), -limx, limx)
    tytz = clamp(f32(view[1] / z), -limy, limy)
    J = [[f32(fx / z), f32(0), f32(0)], [f32(0), f32(fy / z), f32(0)],
         [f32(f32(-fx * txtz) / z), f32(f32(-fy * tytz) / z), f32(0)]]
    Wm = [[f32(u[c * 4 + r]) for r in range(3)] for c in range(3)]
    T = mat3_mul(J, Wm)
    cov = mat3_mul(mat3_mul(T, Sigma), transpose(T))
    a, b, c = f32(cov[0][0] + f32(0.3)), cov[1][0], f32(cov[1][1] + f32(0.3))
    p["cov"] = (a, b, c)
    det = f32(f32(a * c) - f32(b * b))
    if det < f32(0.0001):
        return p
    inv = f32(f32(1) / det)
    p["conic"] = (f32(c * inv), f32(-b * inv), f32(a * inv))
    mid = f32(f32(0.5) * f32(a + c))
    disc = f32(f32(mid * mid) - det)
    l1 = f32(mid + f32(math.sqrt(float(max(f32(0.1), disc)))))
    rr = f32(f32(3) * f32(math.sqrt(float(l1))))
    p["radius"] = f32(min(f32(math.ceil(rr)), f32(512)))
    if p["radius"] <= 0:
        return p
    r = p["radius"]
    minx, miny = max(0, int(f32(sx - r))), max(0, int(f32(sy - r)))
    maxx, maxy = min(int(W) - 1, int(f32(sx + r))), min(int(H) - 1, int(f32(sy + r)))
    if minx > maxx or miny > maxy:
        p["radius"] = f32(0)
        return p
    ntx, nty = int(np.asarray(u[56:58]).view(np.uint32)[0]), int(np.asarray(u[56:58]).view(np.uint32)[1])
    p["tmin"] = (minx // 16, miny // 16)
    p["tmax"] = (min(maxx // 16, ntx - 1), min(maxy // 16, nty - 1))
    if (p["tmax"][0] - p["tmin"][0] + 1) * (p["tmax"][1] - p["tmin"][1] + 1) > 256:
        p["radius"] = f32(0)
        return p
    op = clamp(g[12], -8.0, 8.0)
    p["opacity"] = f32(f32(1) / f32(f32(1) + expf(-op)))
    p["color"] = tuple(clamp(f32(f32(SH_C0 * f32(g[13 + 4 * k])) + f32(0.5)), 0.0, 1.0) for k in range(3))
    return p


def emit_pairs(projs, num_tiles_x):
    """generateTilePairs (tiled_shaders.metal:745-794) in Gaussian order -> list of (key, gid)."""
    out = []
    for gid, p in enumerate(projs):
        if p["radius"] <= 0 or p["opacity"] < f32(0.005):
            continue
        (x0, y0), (x1, y1) = p["tmin"], p["tmax"]
        if x0 > x1 or y0 > y1 or max(x0, x1, y0, y1) > 10000 or (x1 - x0 + 1) * (y1 - y0 + 1) > 256:
            continue
        dk = int(np.asarray([p["depth"]], np.float32).view(np.uint32)[0])
        dk = (~dk & 0xFFFFFFFF) if dk & 0x80000000 else (dk | 0x80000000)
        for ty in range(y0, y1 + 1):
            for tx in range(x0, x1 + 1):
                out.append((((ty * num_tiles_x + tx) << 32) | dk, gid))
    return out


def rasterize(g, u, w, hgt, gt):
    """forward (tiled_rasterizer.mm:275-672 + tiledForward :307-385) and backward (:388-738).

    Returns dict with keys, values, ranges, rgba8, rgb, last_idx, grad (n x 28 float64)."""
    n = g.shape[0]
    u = np.asarray(u, np.float32).copy()
    ntx, nty = (w + 15) // 16, (hgt + 15) // 16
    u.view(np.uint32)[56:59] = [ntx, nty, n]
    projs = [project(g[i], u) for i in range(n)]
    pairs = sorted(emit_pairs(projs, ntx), key=lambda kv: kv[0])  # stable: ties keep gid order
    keys = np.array([k for k, _ in pairs], np.uint64)
    vals = np.array([v for _, v in pairs], np.uint32)
    ranges = np.zeros((ntx * nty, 2), np.uint32)
    tiles = (keys >> np.uint64(32)).astype(np.int64)
    for t in range(ntx * nty):
        lo = int(np.searchsorted(tiles, t, "left"))
        hi = int(np.searchsorted(tiles, t, "right"))
        ranges[t] = (lo, hi - lo)
    rgba = np.zeros((hgt, w), np.uint32)
    rgb = np.zeros((hgt, w, 3), np.float32)
    last = np.full((hgt, w), 0xFFFFFFFF, np.uint32)
    grad = np.zeros((n, 28), np.float64)
    hEps, hMax, hMin = h(0.0001), h(0.99), h(f32(1.0) / f32(255.0))
    for y in range(hgt):
        for x in range(w):
            st, cnt = ranges[(y // 16) * ntx + x // 16]
            px, py = f32(x + 0.5), f32(y + 0.5)
            C = [f16(0)] * 3
            T = f16(1)
            has = False
            for i in range(cnt):
                if not T > hEps:
                    break
                p = projs[vals[st + i]]
                dx, dy = f32(px - p["screen"][0]), f32(py - p["screen"][1])
                c0, c1, c2 = p["conic"]
                if f32(f32(abs(c0) + abs(c1)) + abs(c2)) < f32(0.0001):
                    continue
                q = f32(f32(f32(c0 * dx) * dx) + f32(f32(f32(f32(2) * c1) * dx) * dy))
                q = f32(q + f32(f32(c2 * dy) * dy))
                power = h(f32(f32(-0.5) * q))
                if power > f16(0) or power < f16(-4.5):
                    continue
                G = h(expf(f32(power)))
                alpha = min(f16(h(p["opacity"]) * G), hMax)
                if alpha < hMin:
                    continue
                C = [f16(C[k] + f16(f16(h(p["color"][k]) * alpha) * T)) for k in range(3)]
                T = f16(T * f16(f16(1) - alpha))
                last[y, x] = st + i
                has = True
            if not has:
                last[y, x] = 0xFFFFFFFF
            C = [f16(C[k] + f16(f16(1) * T)) for k in range(3)]
            rgb[y, x] = [f32(c) for c in C]
            q8 = [int(np.rint(f32(min(max(f32(c), f32(0)), f32(1)) * f32(255)))) for c in C]
            rgba[y, x] = q8[0] | (q8[1] << 8) | (q8[2] << 16) | (255 << 24)
    # backward (tiled_shaders.metal:388-738), float32 per term, float64 sums
    for y in range(hgt):
        for x in range(w):
            li = int(last[y, x])
            if li == 0xFFFFFFFF:
                continue
            st, cnt = ranges[(y // 16) * ntx + x // 16]
            px, py = f32(x + 0.5), f32(y + 0.5)
            dl = []
            for k in range(3):
                r = f32(f32((int(rgba[y, x]) >> (8 * k)) & 255) / f32(255))
                t = f32(f32((int(gt[y, x]) >> (8 * k)) & 255) / f32(255))
                d = f32(r - t)
                dl.append(f32((f32(1) if d > 0 else (f32(-1) if d < 0 else f32(0))) / f32(3)))
            end = min(li + 1, int(st + cnt))
            Tf = f32(1)

            def alpha_of(p):
                dx, dy = f32(px - p["screen"][0]), f32(py - p["screen"][1])
                c0, c1, c2 = p["conic"]
                q = f32(f32(f32(c0 * dx) * dx) + f32(f32(f32(f32(2) * c1) * dx) * dy))
                q = f32(q + f32(f32(c2 * dy) * dy))
                pw = f32(f32(-0.5) * q)
                if pw > 0 or pw < f32(-4.5):
                    return None
                G = expf(pw)
                a = f32(min(f32(p["opacity"] * G), f32(0.99)))
                if a < f32(f32(1) / f32(255)):
                    return None
                return a, G, dx, dy
            for s in range(st, end):
                r_ = alpha_of(projs[vals[s]])
                if r_ is None:
                    continue
                tt = f32(Tf * f32(f32(1) - r_[0]))
                if tt < f32(0.0001):
                    break
                Tf = tt
            T = Tf
            acc = [f32(1)] * 3
            fx, fy = f32(u[50]), f32(u[51])
            for s in range(end - 1, int(st) - 1, -1):
                gid = int(vals[s])
                p = projs[gid]
                r_ = alpha_of(p)
                if r_ is None:
                    continue
                a, G, dx, dy = r_
                T = f32(T / f32(max(f32(f32(1) - a), f32(0.0001))))
                wgt = f32(a * T)
                col = p["color"]
                dLc = [f32(0) if (col[k] <= f32(0.01) or col[k] >= f32(0.99)) else f32(dl[k] * wgt)
                       for k in range(3)]
                dd = f32(dl[0] * f32(col[0] - acc[0]))
                dd = f32(dd + f32(dl[1] * f32(col[1] - acc[1])))
                dd = f32(dd + f32(dl[2] * f32(col[2] - acc[2])))
                dA = f32(T * dd)
                acc = [f32(f32(a * col[k]) + f32(f32(f32(1) - a) * acc[k])) for k in range(3)]
                sig = p["opacity"]
                grad[gid, 3] += float(f32(dA * f32(f32(sig * f32(f32(1) - sig)) * G)))
                dG = f32(dA * sig)
                gdx, gdy = f32(G * dx), f32(G * dy)
                c0, c1, c2 = p["conic"]
                ddx = f32(f32(-gdx * c0) - f32(gdy * c1))
                ddy = f32(f32(-gdy * c2) - f32(gdx * c1))
                dSx, dSy = f32(dG * -ddx), f32(dG * -ddy)
                z = p["depth"]
                txtz, tytz = f32(p["vxy"][0] / z), f32(p["vxy"][1] / z)
                dV = [f32(f32(dSx * fx) / z), f32(f32(dSy * fy) / z),
                      f32(f32(f32(f32(-dSx * fx) * txtz) / z) - f32(f32(f32(dSy * fy) * tytz) / z))]
                Wm = [[f32(u[c * 4 + r]) for r in range(3)] for c in range(3)]
                for i in range(3):  # transpose(W) * dV
                    s_ = f32(Wm[i][0] * dV[0])
                    s_ = f32(s_ + f32(Wm[i][1] * dV[1]))
                    s_ = f32(s_ + f32(Wm[i][2] * dV[2]))
                    grad[gid, i] += float(s_)
                grad[gid, 24] += float(dSx)
                grad[gid, 25] += float(dSy)
                for k, off in enumerate((12, 16, 20)):
                    grad[gid, off] += float(f32(dLc[k] * SH_C0))
                dCo = [f32(f32(f32(f32(f32(-0.5) * dG) * G) * dx) * dx),
                       f32(f32(f32(f32(f32(f32(-0.5) * dG) * G) * f32(2)) * dx) * dy),
                       f32(f32(f32(f32(f32(-0.5) * dG) * G) * dy) * dy)]
                ca, cb, cc = p["cov"]
                den = f32(f32(ca * cc) - f32(cb * cb))
                d2i = f32(f32(1) / f32(f32(den * den) + f32(1e-7)))
                dCx = f32(d2i * f32(f32(f32(f32(-cc * cc) * dCo[0]) + f32(f32(f32(f32(2) * cb) * cc) * dCo[1]))
                                    + f32(f32(den - f32(ca * cc)) * dCo[2])))
                dCz = f32(d2i * f32(f32(f32(f32(-ca * ca) * dCo[2]) + f32(f32(f32(f32(2) * ca) * cb) * dCo[1]))
                                    + f32(f32(den - f32(ca * cc)) * dCo[0])))
                dCy = f32(f32(d2i * f32(2)) * f32(f32(f32(f32(cb * cc) * dCo[0])
                                                      - f32(f32(den + f32(f32(f32(2) * cb) * cb)) * dCo[1]))
                                                  + f32(f32(ca * cb) * dCo[2])))
                J = [[f32(fx / z), f32(0), f32(0)], [f32(0), f32(fy / z), f32(0)],
                     [f32(f32(-fx * txtz) / z), f32(f32(-fy * tytz) / z), f32(0)]]
                Tm = mat3_mul(J, Wm)
                D = [[dCx, dCy, f32(0)], [dCy, dCz, f32(0)], [f32(0)] * 3]
                dC3 = mat3_mul(mat3_mul(transpose(Tm), D), Tm)
                gg = g[gid]
                sc = [expf(clamp(gg[4 + k], -5.0, 5.0)) for k in range(3)]
                qr, qx, qy, qz = (f32(v) for v in gg[8:12])
                R = quat_to_mat(qr, qx, qy, qz)
                S = [[sc[0], f32(0), f32(0)], [f32(0), sc[1], f32(0)], [f32(0), f32(0), sc[2]]]
                M = mat3_mul(R, S)
                dM = mat3_mul([[f32(f32(2) * v) for v in col_] for col_ in dC3], M)
                RtdM = mat3_mul(transpose(R), dM)
                for k in range(3):
                    grad[gid, 4 + k] += float(f32(RtdM[k][k] * sc[k]))
                dR = [[f32(dM[c][r] * sc[c]) for r in range(3)] for c in range(3)]
                m = transpose(dR)
                two = f32(2)
                dq0 = f32(two * f32(f32(f32(qz * f32(m[0][1] - m[1][0])) + f32(qy * f32(m[2][0] - m[0][2])))
                                    + f32(qx * f32(m[1][2] - m[2][1]))))
                dq1 = f32(two * f32(f32(f32(f32(qy * f32(m[1][0] + m[0][1])) + f32(qz * f32(m[2][0] + m[0][2])))
                                        + f32(qr * f32(m[1][2] - m[2][1])))
                                    - f32(f32(two * qx) * f32(m[2][2] + m[1][1]))))
                dq2 = f32(two * f32(f32(f32(f32(qx * f32(m[1][0] + m[0][1])) + f32(qr * f32(m[2][0] - m[0][2])))
                                        + f32(qz * f32(m[1][2] + m[2][1])))
                                    - f32(f32(two * qy) * f32(m[2][2] + m[0][0]))))
                dq3 = f32(two * f32(f32(f32(f32(qr * f32(m[0][1] - m[1][0])) + f32(qx * f32(m[2][0] + m[0][2])))
                                        + f32(qy * f32(m[1][2] + m[2][1])))
                                    - f32(f32(two * qz) * f32(m[1][1] + m[0][0]))))
                for k, v in enumerate((dq0, dq1, dq2, dq3)):
                    grad[gid, 8 + k] += float(v)
    return dict(keys=keys, values=vals, ranges=ranges, rgba8=rgba, rgb=rgb, last_idx=last,
                grad=grad, projected=projs)
