#!/usr/bin/env python3
"""Lane-utilisation model of the blend kernels on the bench frame (CPU, from the oracle's forward).

For a sample of tiles, every (list entry, pixel block) the backward evaluates is counted for several
block shapes: a block is evaluated when some pixel of it is in range (entry < the pixel's last
contributor + 1 and 0 <= q <= 9, q = the conic's quadratic form at the pixel centre), and its lanes
are in range / contributing (alpha >= 1/255) or idle. The current kernels evaluate 8x8 bands (64
lanes). Smaller blocks evaluate fewer idle lanes; this script says how many.

  python scripts/lane_util.py [--tiles 400] [--gaussians 1000000]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=400)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=3)
    args = ap.parse_args()
    from gaussiansplatting_amd import scene
    from oracle import oracle
    w, h = 1920, 1080
    g = scene.synthetic_gaussians(args.gaussians, args.seed, w, h)
    u = scene.rig_uniforms(0, w, h)
    f = oracle.forward(g, u, w, h, threads=os.cpu_count() or 8)
    pr = f.projected
    tx, ty = (w + 15) // 16, (h + 15) // 16
    rng = np.random.default_rng(0)
    tiles = rng.choice(tx * ty, size=min(args.tiles, tx * ty), replace=False)
    shapes = [(8, 8), (8, 4), (4, 4), (4, 2), (2, 2)]
    bw = {s: dict(blocks=0, lanes_in=0, lanes_con=0) for s in shapes}
    fw = {s: dict(blocks=0, lanes_in=0) for s in shapes}
    splats_sel = 0
    for t in tiles:
        start, cnt = f.ranges[t]
        if cnt == 0:
            continue
        vals = f.values[start:start + cnt]
        X, Y = (t % tx) * 16, (t // tx) * 16
        yy, xx = np.mgrid[0:16, 0:16]
        px = (X + xx + 0.5).astype(np.float32)
        py = (Y + yy + 0.5).astype(np.float32)
        inside = (X + xx < w) & (Y + yy < h)
        li = np.full((16, 16), 0xFFFFFFFF, np.uint32)
        ys, xs = np.clip(Y + yy, 0, h - 1), np.clip(X + xx, 0, w - 1)
        li = np.where(inside, f.last_idx[ys, xs], 0xFFFFFFFF)
        last = np.where(li == 0xFFFFFFFF, 0, li.astype(np.int64) + 1)  # exclusive
        sidx = start + np.arange(cnt, dtype=np.int64)
        rec = pr[vals]
        sx, sy = rec[:, 0, None, None], rec[:, 1, None, None]
        c0, c1, c2 = rec[:, 2, None, None], rec[:, 3, None, None], rec[:, 4, None, None]
        op = rec[:, 6, None, None]
        dx, dy = px[None] - sx, py[None] - sy
        q = c0 * dx * dx + 2.0 * c1 * dx * dy + c2 * dy * dy
        inr = (q >= 0) & (q <= 9)
        act_b = inr & (sidx[:, None, None] < last[None])
        alpha = np.minimum(op * np.exp(-0.5 * q), 0.99)
        con_b = act_b & (alpha >= 1.0 / 255.0)
        # forward: a pixel takes entries until its T drops to 1e-4 (float model of the half blend)
        a_f = np.where(inr & (alpha >= 1.0 / 255.0), alpha, 0.0)
        Tcum = np.cumprod(1.0 - a_f, axis=0)
        Tbefore = np.concatenate([np.ones((1, 16, 16)), Tcum[:-1]], axis=0)
        act_f = inr & (Tbefore > 1e-4) & inside[None]
        splats_sel += int(act_b.reshape(cnt, -1).any(1).sum())
        for (bwid, bhei) in shapes:
            ab = act_b.reshape(cnt, 16 // bhei, bhei, 16 // bwid, bwid)
            cb = con_b.reshape(cnt, 16 // bhei, bhei, 16 // bwid, bwid)
            af = act_f.reshape(cnt, 16 // bhei, bhei, 16 // bwid, bwid)
            hit = ab.any(axis=(2, 4))
            bw[(bwid, bhei)]["blocks"] += int(hit.sum())
            bw[(bwid, bhei)]["lanes_in"] += int(ab.sum())
            bw[(bwid, bhei)]["lanes_con"] += int(cb.sum())
            hf = af.any(axis=(2, 4))
            fw[(bwid, bhei)]["blocks"] += int(hf.sum())
            fw[(bwid, bhei)]["lanes_in"] += int(af.sum())
    cur, exact, box, ent, oct_, half_ = forward_steps(f, pr, tiles, w, h, tx)
    print(f"forward pair steps: 8x8 band lists {cur}, 4x4 quadrant groups exact cull {exact} "
          f"({exact / cur:.3f}), box cull {box} ({box / cur:.3f}), 4x2 groups {oct_} ({oct_ / cur:.3f}), "
          f"8x4 halves {half_} ({half_ / cur:.3f}); band entries {ent}")
    v0, v1, v1p, v2, v1h = backward_costs(f, pr, tiles, w, h, tx)
    print(f"backward VALU model: today {v0:.3e}, band-first quadrant items {v1:.3e} ({v1 / v0:.3f}), "
          f"with pair reductions {v1p:.3e} ({v1p / v0:.3f}), entry-first groups {v2:.3e} ({v2 / v0:.3f}), "
          f"half-band groups {v1h:.3e} ({v1h / v0:.3f})")
    print(f"tiles sampled {len(tiles)}, pairs {f.num_pairs}, backward selected splats {splats_sel}")
    for s in shapes:
        b, ff = bw[s], fw[s]
        lanes = s[0] * s[1]
        print(f"block {s[0]}x{s[1]}: backward blocks {b['blocks']:9d} lane-evals {b['blocks'] * lanes:11d} "
              f"in-range {b['lanes_in'] / max(1, b['blocks'] * lanes):.3f} contributing "
              f"{b['lanes_con'] / max(1, b['blocks'] * lanes):.3f} | forward blocks {ff['blocks']:9d} "
              f"lane-evals {ff['blocks'] * lanes:11d} in-range {ff['lanes_in'] / max(1, ff['blocks'] * lanes):.3f}")
    return 0



def forward_steps(f, pr, tiles, w, h, tx):
    """Pair steps of the forward blend per (tile, band, chunk): today ceil(nsel / 2) (one list per
    8x8 band wave), with 4x4 quadrant groups max_g ceil(n_g / 2) (each 16-lane group walks its own
    list), for an exact quadrant cull and for a box cull (the conservative extents)."""
    cur = exact = box = oct_ = half_ = 0
    ent = 0
    for t in tiles:
        start, cnt = f.ranges[t]
        if cnt == 0:
            continue
        vals = f.values[start:start + cnt]
        X, Y = (t % tx) * 16, (t // tx) * 16
        yy, xx = np.mgrid[0:16, 0:16]
        px = (X + xx + 0.5).astype(np.float64)
        py = (Y + yy + 0.5).astype(np.float64)
        inside = (X + xx < w) & (Y + yy < h)
        rec = pr[vals].astype(np.float64)
        sx, sy = rec[:, 0, None, None], rec[:, 1, None, None]
        c0, c1, c2 = rec[:, 2, None, None], rec[:, 3, None, None], rec[:, 4, None, None]
        op = rec[:, 6, None, None]
        K = np.minimum(9.01, 2 * np.log(255 * np.maximum(op, 1e-30)) + 0.02)
        dx, dy = px[None] - sx, py[None] - sy
        q = c0 * dx * dx + 2.0 * c1 * dx * dy + c2 * dy * dy
        geo = (q >= 0) & (q <= K)
        alpha = np.minimum(op * np.exp(-0.5 * q), 0.99)
        a_f = np.where((q >= 0) & (q <= 9) & (alpha >= 1.0 / 255.0), alpha, 0.0)
        Tcum = np.cumprod(1.0 - a_f, axis=0)
        Tb = np.concatenate([np.ones((1, 16, 16)), Tcum[:-1]], axis=0)
        alive = (Tb > 1e-4) & inside[None]
        # box extents (cull_extents)
        Kc = K[:, 0, 0]
        A, C, B = c0[:, 0, 0], c2[:, 0, 0], np.abs(c1[:, 0, 0])
        D = A * C - B * B
        ex = np.where(D > 0, np.sqrt(np.maximum(Kc * C / np.where(D > 0, D, 1), 0)) + 1e-3, np.inf)
        ey = np.where(D > 0, np.sqrt(np.maximum(Kc * A / np.where(D > 0, D, 1), 0)) + 1e-3, np.inf)
        s_x, s_y = rec[:, 0], rec[:, 1]
        for b in range(4):
            bx, by = (b % 2) * 8, (b // 2) * 8
            g_b = geo[:, by:by + 8, bx:bx + 8]
            al_b = alive[:, by:by + 8, bx:bx + 8]
            for c0_ in range(0, cnt, 64):
                if not al_b[c0_].any():
                    break
                sl = slice(c0_, min(c0_ + 64, cnt))
                hit = g_b[sl].any(axis=(1, 2))
                ent += hit.sum()
                cur += (int(hit.sum()) + 1) // 2
                ne, nb = [], []
                for qd in range(4):
                    qx, qy = (qd % 2) * 4, (qd // 2) * 4
                    qe = g_b[sl, qy:qy + 4, qx:qx + 4].any(axis=(1, 2))
                    ne.append(int(qe.sum()))
                    x0, x1 = X + bx + qx + 0.5, X + bx + qx + 3.5
                    y0, y1 = Y + by + qy + 0.5, Y + by + qy + 3.5
                    qb = hit & ~((s_x[sl] + ex[sl] < x0) | (s_x[sl] - ex[sl] > x1) |
                                 (s_y[sl] + ey[sl] < y0) | (s_y[sl] - ey[sl] > y1))
                    nb.append(int(qb.sum()))
                exact += max((n + 1) // 2 for n in ne)
                box += max((n + 1) // 2 for n in nb)
                # eight 8-lane groups of 4x2 blocks
                n8 = []
                for qd in range(8):
                    qx, qy = (qd % 2) * 4, (qd // 2) * 2
                    n8.append(int(g_b[sl, qy:qy + 2, qx:qx + 4].any(axis=(1, 2)).sum()))
                oct_ += max((n + 1) // 2 for n in n8)
                # two 32-lane groups of 8x4 halves
                n2 = [int(g_b[sl, 0:4, :].any(axis=(1, 2)).sum()), int(g_b[sl, 4:8, :].any(axis=(1, 2)).sum())]
                half_ += max((n + 1) // 2 for n in n2)
    return cur, exact, box, ent, oct_, half_


def backward_costs(f, pr, tiles, w, h, tx, ev=49.0, red64=23.0, red16=33.0, red16_pair=28.5):
    """VALU model of the backward per tile (one wave, 4 pixels per lane, reverse list in 64-entry
    chunks up to the last contributor). V0 (today): per selected entry, one 64-lane evaluation per
    8x8 band it reaches + a 64-lane reduction. V1: 16-lane groups own one 4x4 quadrant of every band;
    per (chunk, band) each group walks the entries that reach its quadrant (items), one 16-lane
    reduction per item. V2: each group walks the entries that reach any of its quadrants; per step
    the wave evaluates the union of the groups' current band masks, one 16-lane reduction per step."""
    v0 = v1 = v1p = v2 = v1h = 0.0
    for t in tiles:
        start, cnt = f.ranges[t]
        if cnt == 0:
            continue
        vals = f.values[start:start + cnt]
        X, Y = (t % tx) * 16, (t // tx) * 16
        yy, xx = np.mgrid[0:16, 0:16]
        px = (X + xx + 0.5).astype(np.float64)
        py = (Y + yy + 0.5).astype(np.float64)
        inside = (X + xx < w) & (Y + yy < h)
        ys, xs = np.clip(Y + yy, 0, h - 1), np.clip(X + xx, 0, w - 1)
        li = np.where(inside, f.last_idx[ys, xs], 0xFFFFFFFF)
        last = np.where(li == 0xFFFFFFFF, 0, li.astype(np.int64) + 1)
        end_max = max(int(last.max()), int(start))
        n_used = end_max - int(start)
        if n_used <= 0:
            continue
        sidx = start + np.arange(n_used, dtype=np.int64)
        rec = pr[vals[:n_used]].astype(np.float64)
        sx, sy = rec[:, 0, None, None], rec[:, 1, None, None]
        c0, c1, c2 = rec[:, 2, None, None], rec[:, 3, None, None], rec[:, 4, None, None]
        op = rec[:, 6, None, None]
        K = np.minimum(9.01, 2 * np.log(255 * np.maximum(op, 1e-30)) + 0.02)
        dx, dy = px[None] - sx, py[None] - sy
        q = c0 * dx * dx + 2.0 * c1 * dx * dy + c2 * dy * dy
        geo = (q >= 0) & (q <= K)
        band_end = [int(last[(b // 2) * 8:(b // 2) * 8 + 8, (b % 2) * 8:(b % 2) * 8 + 8].max()) for b in range(4)]
        # hit[e, band, quad]
        hit = np.zeros((n_used, 4, 4), bool)
        for b in range(4):
            bx, by = (b % 2) * 8, (b // 2) * 8
            ok = sidx < band_end[b]
            for qd in range(4):
                qx, qy = (qd % 2) * 4, (qd // 2) * 4
                hit[:, b, qd] = ok & geo[:, by + qy:by + qy + 4, bx + qx:bx + qx + 4].any(axis=(1, 2))
        bandhit = hit.any(axis=2)  # [e, band]
        for c in range(0, n_used, 64):
            sl = slice(c, min(c + 64, n_used))
            bh = bandhit[sl]
            sel = bh.any(axis=1)
            v0 += ev * bh.sum() + red64 * sel.sum()
            hq = hit[sl]  # [e, band, quad]
            for b in range(4):
                n = hq[:, b, :].sum(axis=0)  # per quad
                steps = int(n.max())
                v1 += steps * (ev + red16)
                v1p += steps * (ev + red16_pair)
            # V1h: two 32-lane groups, the top and bottom 8x4 halves of band b, each walking its
            # half's entries; one 32-lane reduction per step and group (24 VALU for both)
            for b in range(4):
                top = (hq[:, b, 0] | hq[:, b, 1]).sum()
                bot = (hq[:, b, 2] | hq[:, b, 3]).sum()
                v1h += max(top, bot) * (ev + 24.0)
            # V2: group g's entries: any band hit for quad g
            lists = [np.nonzero(hq[:, :, g].any(axis=1))[0] for g in range(4)]
            steps = max(len(l) for l in lists)
            for s_ in range(steps):
                union = np.zeros(4, bool)
                for g in range(4):
                    if s_ < len(lists[g]):
                        union |= hq[lists[g][s_], :, g]
                v2 += ev * union.sum() + red16
    return v0, v1, v1p, v2, v1h


if __name__ == "__main__":
    sys.exit(main())
