"""Adam optimizer and opacity reset.

CPU: the oracle's restatement of adamStep (shaders.metal:536-713, over the reference's own state
layout, optimizer.mm:46-73) against an independent numpy float32 restatement — bit-exact.
GPU: the HIP kernel (one 96-B moment record per Gaussian) against the oracle — bit-exact for the
Gaussians and both moments over several steps, the skip rules, the momentum resets, the moments
following a density apply, and the opacity reset."""
from __future__ import annotations

import numpy as np
import pytest

from gaussiansplatting_amd import scene

LRS = (0.00016, 0.005, 0.001, 0.025, 0.0025)  # mtl_engine.mm:1060-1069 (opacity 0.025)
f32 = np.float32


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    g = scene.synthetic_gaussians(n, seed, 64, 48)
    # non-zero higher SH so the +-2 clamp and the zero-gradient path both show
    g[:, 13:25] += rng.normal(0, 1.5, (n, 12)).astype(np.float32)
    d = np.zeros((n, 28), np.float32)
    for o in (0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 16, 20):
        d[:, o] = rng.normal(0, 0.3, n).astype(np.float32)
    d[:, 12:24] += (rng.random((n, 12)) < 0.2) * rng.normal(0, 2.0, (n, 12)).astype(np.float32)
    # edge cases: NaN / inf gradients (skipped), corrupted position (skipped), huge step (limited),
    # a rotation that collapses to zero length (reset to identity)
    d[0, 0] = np.nan
    d[1, 3] = np.inf
    d[2, 12] = np.nan
    g[3, 0] = 2e6
    d[4, 0:3] = 0.5
    g[5, 8:12] = 0.0
    d[5, 8:12] = 0.0
    return g, d


def _np_adam(g, d, st, lrs, t):
    """Independent numpy float32 restatement of adamStep (vectorised, same operation order)."""
    b1, b2, eps, clip = f32(0.9), f32(0.999), f32(1e-8), f32(0.5)
    bc1 = f32(1.0) - f32(float(b1) ** t)
    bc2 = f32(1.0) - f32(float(b2) ** t)
    one = f32(1.0)
    skip = (np.isnan(d[:, 0]) | np.isnan(d[:, 3]) | np.isnan(d[:, 12]) | np.isinf(d[:, 0]) |
            np.isinf(d[:, 3]) | np.isnan(g[:, 0]) | np.isinf(g[:, 0]) | (np.abs(g[:, 0]) > f32(1e6)))
    ok = ~skip

    def upd(grad, m, v, lr):
        gc = np.minimum(np.maximum(grad, -clip), clip)
        m2 = b1 * m + (one - b1) * gc
        v2 = b2 * v + (one - b2) * gc * gc
        return m2, v2, f32(lr) * (m2 / bc1) / (np.sqrt(v2 / bc2) + eps)

    G = g.copy()
    M, V = st["m"].copy(), st["v"].copy()
    # position
    m2, v2, u = upd(d[:, 0:3], M[:, 0:3], V[:, 0:3], lrs[0])
    mag = np.sqrt(u[:, 0] * u[:, 0] + u[:, 1] * u[:, 1] + u[:, 2] * u[:, 2])
    big = mag > f32(0.1)
    u = np.where(big[:, None], u * (f32(0.1) / np.where(big, mag, one))[:, None], u)
    npos = g[:, 0:3] - u
    sane = ~np.isnan(npos).any(1) & (np.abs(npos) < f32(1e6)).all(1)
    G[:, 0:3] = np.where(sane[:, None], npos, g[:, 0:3])
    M[:, 0:3], V[:, 0:3] = m2, v2
    # scale
    m2, v2, u = upd(d[:, 4:7], M[:, 4:7], V[:, 4:7], lrs[1])
    G[:, 4:7] = np.minimum(np.maximum(g[:, 4:7] - u, f32(-4)), f32(4))
    M[:, 4:7], V[:, 4:7] = m2, v2
    # rotation
    m2, v2, u = upd(d[:, 8:12], M[:, 8:12], V[:, 8:12], lrs[2])
    nr = g[:, 8:12] - u
    ln = np.sqrt(nr[:, 0] * nr[:, 0] + nr[:, 1] * nr[:, 1] + nr[:, 2] * nr[:, 2] + nr[:, 3] * nr[:, 3])
    okr = ln > f32(0.001)
    ident = np.array([1, 0, 0, 0], np.float32)
    G[:, 8:12] = np.where(okr[:, None], nr / np.where(okr, ln, one)[:, None], ident)
    M[:, 8:12], V[:, 8:12] = m2, v2
    # opacity
    m2, v2, u = upd(d[:, 3], M[:, 3], V[:, 3], lrs[3])
    G[:, 12] = np.minimum(np.maximum(g[:, 12] - u, f32(-8)), f32(8))
    M[:, 3], V[:, 3] = m2, v2
    # sh
    m2, v2, u = upd(d[:, 12:24], M[:, 12:24], V[:, 12:24], lrs[4])
    G[:, 13:25] = np.minimum(np.maximum(g[:, 13:25] - u, f32(-2)), f32(2))
    M[:, 12:24], V[:, 12:24] = m2, v2
    G = np.where(ok[:, None], G, g)
    st["m"] = np.where(ok[:, None], M, st["m"])
    st["v"] = np.where(ok[:, None], V, st["v"])
    return G


def test_oracle_adam_matches_numpy():
    from oracle import oracle
    n = 600
    g, d = _inputs(n, 7)
    st = oracle.AdamState(n)
    ref = {"m": np.zeros((n, 24), np.float32), "v": np.zeros((n, 24), np.float32)}
    go, gn = g.copy(), g.copy()
    with np.errstate(invalid="ignore", over="ignore"):
        for t in range(1, 5):
            oracle.adam_step(go, d, st, LRS)
            gn = _np_adam(gn, d, ref, LRS, t)
            assert np.array_equal(go.view(np.uint32), gn.view(np.uint32)), f"Gaussians differ at t={t}"
            assert np.array_equal(st.records("m").view(np.uint32), ref["m"].view(np.uint32))
            assert np.array_equal(st.records("v").view(np.uint32), ref["v"].view(np.uint32))
    # the edge cases did what the reference does
    assert np.array_equal(go[0].view(np.uint32), g[0].view(np.uint32))   # NaN gradient: skipped
    assert np.array_equal(go[3].view(np.uint32), g[3].view(np.uint32))   # corrupted: skipped
    assert np.array_equal(go[5, 8:12], np.array([1, 0, 0, 0], np.float32))  # zero length: identity
    assert np.all(np.abs(go[6:, 13:25]) <= 2.0)  # updated rows are clamped to +-2


def test_oracle_opacity_reset():
    from oracle import oracle
    g = scene.synthetic_gaussians(100, 3, 32, 32)
    g[::3, 12] = -6.0
    want = np.minimum(g[:, 12], np.float32(-4.6))
    oracle.opacity_reset(g, -4.6)
    assert np.array_equal(g[:, 12], want)


@pytest.mark.gpu
def test_gpu_adam_parity(dev):
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer
    from oracle import oracle
    n = 5000
    g, d = _inputs(n, 11)
    opt = AdamOptimizer(n)
    gt_ = torch.from_numpy(g.copy()).to(dev)
    dt_ = torch.from_numpy(d).to(dev)
    st = oracle.AdamState(n)
    go = g.copy()
    with np.errstate(invalid="ignore", over="ignore"):
        for t in range(1, 6):
            opt.step(gt_, dt_, LRS)
            oracle.adam_step(go, d, st, LRS)
            torch.cuda.synchronize()
            gg = gt_.cpu().numpy()
            assert np.array_equal(gg.view(np.uint32), go.view(np.uint32)), f"Gaussians differ at t={t}"
            m, v = opt.state(n)
            assert np.array_equal(m.view(np.uint32), st.records("m").view(np.uint32)), f"m differs at t={t}"
            assert np.array_equal(v.view(np.uint32), st.records("v").view(np.uint32)), f"v differs at t={t}"
    assert opt.timestep == 5
    # momentum resets (optimizer.mm:137-147)
    opt.reset_opacity_momentum(n)
    opt.reset_scale_momentum(n)
    m, v = opt.state(n)
    assert not m[:, 3].any() and not v[:, 3].any() and not m[:, 4:7].any() and not v[:, 4:7].any()
    assert m[:, 0:3].any()
    opt.reset_state_for_new_gaussians(4000, n)
    m, v = opt.state(n)
    assert not m[4000:].any() and m[:4000, 0:3].any()
    opt.reset()
    m, v = opt.state(n)
    assert not m.any() and not v.any() and opt.timestep == 0


@pytest.mark.gpu
def test_gpu_adam_rows_cold_lanes(dev):
    """The row-path update touches only the moment quads of the fields with rasterizer gradients
    while every other moment lane is zero (gs_adam.hpp mom_sh_lane), and loads no moments for a
    Gaussian whose records were never non-zero. Bit-exact against the oracle: rows steps from a
    fresh state (the higher SH only clamped; a block of Gaussians without gradients until the last); a records step with non-zero higher-SH
    gradients and then rows steps (those lanes decay); a written state with non-zero higher-SH lanes
    and then a rows step (equal to the records path on the same state); and read_state / write_state
    round trips in the reference's lane order."""
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer
    from oracle import oracle
    n = 3000
    g, d = _inputs(n, 23)
    rf = scene.ROW_FIELDS
    rows = torch.from_numpy(np.ascontiguousarray(d[:, rf])).to(dev)
    d_rows = np.zeros_like(d)
    d_rows[:, rf] = d[:, rf]  # what a rows step sees as its records
    with np.errstate(invalid="ignore", over="ignore"):
        for records_first in (False, True):
            opt = AdamOptimizer(n)
            gt_ = torch.from_numpy(g.copy()).to(dev)
            st = oracle.AdamState(n)
            go = g.copy()
            if records_first:
                opt.step(gt_, torch.from_numpy(d).to(dev), LRS)
                oracle.adam_step(go, d, st, LRS)
            for t in range(3):
                # the first 700 Gaussians get no gradient before the last step: zero moments that
                # the update does not load (gs_adam.hpp live flags) until a gradient reaches them
                dz = d_rows.copy()
                if t < 2:
                    dz[:700] = 0.0
                opt.step_rows(gt_, torch.from_numpy(np.ascontiguousarray(dz[:, rf])).to(dev), LRS)
                oracle.adam_step(go, dz, st, LRS)
                torch.cuda.synchronize()
                label = f"records_first={records_first} rows step {t}"
                assert np.array_equal(gt_.cpu().numpy().view(np.uint32), go.view(np.uint32)), label
                m, v = opt.state(n)
                assert np.array_equal(m.view(np.uint32), st.records("m").view(np.uint32)), label
                assert np.array_equal(v.view(np.uint32), st.records("v").view(np.uint32)), label
            if records_first:
                assert m[:, [13, 14, 15, 17, 18, 19, 21, 22, 23]].any()  # the higher-SH lanes carry moments
        # a written state with non-zero higher-SH lanes: the rows step equals the records step
        rng = np.random.default_rng(5)
        ms = rng.normal(0, 0.1, (n, 24)).astype(np.float32)
        vs = np.abs(rng.normal(0, 0.1, (n, 24))).astype(np.float32)
        ms[:, 7] = vs[:, 7] = 0.0
        outs = []
        for use_rows in (True, False):
            opt = AdamOptimizer(n)
            opt.set_state(torch.from_numpy(ms).to(dev), torch.from_numpy(vs).to(dev), n)
            m0, v0 = opt.state(n)
            assert np.array_equal(m0, ms) and np.array_equal(v0, vs)  # the round trip
            gt_ = torch.from_numpy(g.copy()).to(dev)
            if use_rows:
                opt.step_rows(gt_, rows, LRS)
            else:
                opt.step(gt_, torch.from_numpy(d_rows).to(dev), LRS)
            torch.cuda.synchronize()
            outs.append((gt_.cpu().numpy(),) + opt.state(n))
        for a, b in zip(*outs):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
def test_gpu_adam_follows_density_apply(dev):
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer, DensityController
    from oracle import oracle
    n, w, h = 3000, 96, 64
    g = scene.synthetic_gaussians(n, 5, w, h)
    d = np.zeros((n, 28), np.float32)
    rng = np.random.default_rng(2)
    d[:, 0:3] = rng.normal(0, 0.2, (n, 3))
    d[:, 24:26] = rng.normal(0, 0.01, (n, 2))  # viewspace gradients drive densification
    d[:, 3] = rng.normal(0, 0.2, n)
    gt_ = torch.from_numpy(g.copy()).to(dev)
    dt_ = torch.from_numpy(d).to(dev)
    opt = AdamOptimizer(n)
    opt.step(gt_, dt_, LRS)
    m0, v0 = opt.state(n)
    dc = DensityController()
    dc.set_scene_extent(2.0)
    dc.reset_accumulator(n)
    dc.accumulate_gradients(dt_)
    new, stats = dc.apply(gt_, 600, focal_length=float(w), image_width=float(w), avg_depth=6.0, seed=9)
    n_out = int(new.shape[0])
    assert stats["num_cloned"] + stats["num_split"] + stats["num_pruned"] > 0
    opt.follow_density(dc, n, n_out)
    m1, v1 = opt.state(n_out)
    # expected: walk the markers exactly as density_control.mm:392-482 emits
    _, marker, _ = oracle.density_apply(g, *_accum(d, n), 600, 2.0, float(w), float(w), 6.0, 9)
    em = np.zeros((n_out, 24), np.float32)
    ev = np.zeros((n_out, 24), np.float32)
    o = 0
    for i, mk in enumerate(marker):
        if mk == 1:
            continue
        if mk == 0:
            em[o], ev[o] = m0[i], v0[i]
            o += 1
        elif mk == 2:
            em[o], ev[o] = m0[i], v0[i]
            o += 2
        else:
            o += 2
    assert o == n_out
    assert np.array_equal(m1, em) and np.array_equal(v1, ev)


def _accum(d, n):
    from oracle import oracle
    acc = np.zeros(n, np.float32)
    cnt = np.zeros(n, np.uint32)
    pos = np.zeros((n, 3), np.float32)
    oracle.density_accumulate(d, acc, cnt, pos)
    return acc, cnt


@pytest.mark.gpu
def test_gpu_opacity_reset(dev):
    import torch

    from gaussiansplatting_amd.rasterizer import opacity_reset
    from oracle import oracle
    g = scene.synthetic_gaussians(10000, 4, 64, 64)
    t = torch.from_numpy(g.copy()).to(dev)
    opacity_reset(t, -4.6)
    oracle.opacity_reset(g, -4.6)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy().view(np.uint32), g.view(np.uint32))
