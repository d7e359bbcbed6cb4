"""CPU tests of the oracle: pinned against the committed golden fixtures, the reference's own runtime
self-checks (tiled_rasterizer.mm:577-636, gpu_sort.mm:653-671) as hard assertions, and the
density-control restatement's invariants."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from gaussiansplatting_amd import scene

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _oracle():
    from oracle import oracle
    return oracle


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_golden_small_full_buffers():
    o = _oracle()
    d = np.load(os.path.join(GOLDEN, "golden_small.npz"))
    g, u, gt = d["gaussians"], d["uniforms"], d["gt"]
    f = o.forward(g, u, 64, 64, threads=2)
    for k in ("keys", "values", "ranges", "last_idx", "rgba8"):
        assert np.array_equal(getattr(f, k), d[k]), k
    assert np.array_equal(f.rgb.view(np.uint32), d["rgb"].view(np.uint32))
    assert np.array_equal(f.projected.view(np.uint32), d["projected"].view(np.uint32))
    gr, ab, nz = o.backward(g, f, f.rgba8, gt, threads=2)
    live = [off for _, off in scene.GRAD_FIELDS]
    np.testing.assert_allclose(gr[:, live], d["grad"], rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(ab[:, live], d["grad_abs"], rtol=1e-12, atol=1e-300)


def test_golden_cfg1_hashes():
    o = _oracle()
    d = np.load(os.path.join(GOLDEN, "golden_cfg1.npz"))
    c = scene.CONFIGS[1]
    g = scene.synthetic_gaussians(c["n"], c["seed"], c["width"], c["height"])
    # the generator is part of the contract: regenerated inputs equal the committed ones
    assert np.array_equal(g.view(np.uint32), d["gaussians"].view(np.uint32))
    assert np.array_equal(scene.make_uniforms(256, 256).view(np.uint32), d["uniforms"].view(np.uint32))
    f = o.forward(d["gaussians"], d["uniforms"], 256, 256)
    assert f.num_pairs == int(d["num_pairs"])
    assert sha(f.keys) == str(d["sha_keys"])
    assert sha(f.values) == str(d["sha_values"])
    assert sha(f.ranges) == str(d["sha_ranges"])
    assert sha(f.last_idx) == str(d["sha_last_idx"])
    assert sha(f.rgba8) == str(d["sha_rgba8"])
    assert sha(f.rgb) == str(d["sha_rgb"])
    assert sha(f.projected) == str(d["sha_projected"])


@pytest.mark.parametrize("n,w,h,seed", [(3000, 100, 75, 1), (20000, 320, 180, 2)])
def test_reference_self_checks(n, w, h, seed):
    """tiled_rasterizer.mm:577-636: ranges contiguous, coverage == pair count; keys monotone."""
    o = _oracle()
    g = scene.synthetic_gaussians(n, seed, w, h)
    f = o.forward(g, scene.make_uniforms(w, h), w, h)
    P = f.num_pairs
    assert P > 0
    assert np.all(np.diff(f.keys.astype(np.uint64)) >= 0) if P > 1 else True
    assert int(f.ranges[:, 1].sum()) == P
    nz = f.ranges[f.ranges[:, 1] > 0]
    assert np.array_equal(nz[1:, 0], nz[:-1, 0] + nz[:-1, 1])  # contiguous
    tiles = (f.keys >> np.uint64(32)).astype(np.int64)
    for t in np.unique(tiles)[:50]:
        s, cnt = f.ranges[t]
        assert np.all(tiles[s:s + cnt] == t)
    # every pair comes from its Gaussian's tile rect
    pr = f.projected.view(scene.PROJECTED_DTYPE).reshape(-1)
    tx = tiles % ((w + 15) // 16)
    ty = tiles // ((w + 15) // 16)
    v = f.values
    assert np.all((pr["tile_min_x"][v] <= tx) & (tx <= pr["tile_max_x"][v]))
    assert np.all((pr["tile_min_y"][v] <= ty) & (ty <= pr["tile_max_y"][v]))
    # last contributor lies inside its tile's range
    li = f.last_idx
    ok = li != 0xFFFFFFFF
    yy, xx = np.nonzero(ok)
    t = (yy // 16) * ((w + 15) // 16) + xx // 16
    assert np.all(li[ok] >= f.ranges[t, 0]) and np.all(li[ok] < f.ranges[t, 0] + f.ranges[t, 1])


def test_sort_is_stable_lsd():
    o = _oracle()
    rng = np.random.default_rng(3)
    keys = (rng.integers(0, 50, 5000).astype(np.uint64) << np.uint64(32)) | rng.integers(0, 8, 5000).astype(np.uint64)
    vals = np.arange(5000, dtype=np.uint32)
    k, v = o.sort_pairs(keys, vals, threads=3)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(k, keys[order]) and np.array_equal(v, vals[order])


def test_backward_shadow_matches_float_sums():
    """backward_shadow's float sums are backward()'s bit for bit; its fp64 shadow lies within the
    float terms' own rounding noise (summed |float - fp64| per field) of them; a huge splat whose
    float dSigma chain overflows (NaN) has a finite shadow."""
    o = _oracle()
    w = h = 96
    g = scene.synthetic_gaussians(600, 4, w, h)
    g[:8, 4:7] = 8.0  # clamped at the maximum log-scale: radius beyond the view
    u = scene.make_uniforms(w, h)
    gt = scene.synthetic_ground_truth(4, 0, w, h)
    f = o.forward(g, u, w, h, threads=2)
    gr, ab, nz = o.backward(g, f, f.rgba8, gt, threads=2)
    gr2, sh = o.backward_shadow(g, f, f.rgba8, gt, threads=2)
    assert np.array_equal(gr, gr2, equal_nan=True)
    assert np.all(np.isfinite(sh))
    fin = np.isfinite(gr)
    assert np.all(np.abs(gr - sh)[fin] <= nz[fin] * (1 + 1e-9) + 1e-300)


def test_empty_scene_returns_before_rendering():
    o = _oracle()
    g = scene.synthetic_gaussians(100, 1, 32, 32)
    g[:, 2] = -5.0
    f = o.forward(g, scene.make_uniforms(32, 32), 32, 32)
    assert f.num_pairs == 0
    assert np.all(f.last_idx == 0xFFFFFFFF) and np.all(f.ranges == 0)
    assert np.all(f.rgba8 == 0)  # untouched


def test_density_accumulate_rules():
    o = _oracle()
    n = 6
    grads = np.zeros((n, 28), np.float32)
    grads[0, 24:26] = [3.0, 4.0]            # |g| = 5 -> clamped to 1
    grads[1, 24:26] = [0.0, 0.0]            # zero -> not counted
    grads[2, 24:26] = [np.nan, 1.0]         # NaN -> not counted
    grads[3, 24:26] = [1e-3, 0.0]
    grads[3, 0:3] = [1.0, 2.0, 3.0]
    grads[4, 24:26] = [np.inf, 0.0]         # inf clamps to 1 (std::min) and is counted
    acc = np.zeros(n, np.float32)
    cnt = np.zeros(n, np.uint32)
    pos = np.zeros((n, 3), np.float32)
    o.density_accumulate(grads, acc, cnt, pos)
    assert acc[0] == 1.0 and cnt[0] == 1
    assert cnt[1] == 0 and cnt[2] == 0
    assert np.isclose(acc[3], 1e-3) and np.array_equal(pos[3], [1, 2, 3])
    assert acc[4] == 1.0 and cnt[4] == 1


def test_density_apply_rules():
    o = _oracle()
    g = scene.synthetic_gaussians(400, 9, 64, 64)
    acc = np.full(400, 0.01, np.float32)
    cnt = np.ones(400, np.uint32)
    acc[:100] = 0.0                          # below the gradient threshold: kept
    g[100:110, 12] = -8.0                    # sigmoid < 0.005: pruned
    out, mk, st = o.density_apply(g, acc, cnt, 600, 1.0, 64.0, 64.0, 5.0, seed=4)
    assert np.all(mk[:100][g[:100, 12] > -5.0] == 0)
    assert np.all(mk[100:110] == 1)
    assert st["num_pruned"] >= 10 and st["num_cloned"] + st["num_split"] > 0
    assert out.shape[0] == 400 - st["num_pruned"] + st["num_cloned"] + st["num_split"]
    # splits: two children symmetric about the parent, log-scale reduced by ln(1.6)
    idx = np.nonzero(mk == 3)[0]
    if idx.size:
        slots = np.cumsum([0] + [0 if m == 1 else (1 if m == 0 else 2) for m in mk])
        i = idx[0]
        c1, c2 = out[slots[i]], out[slots[i] + 1]
        np.testing.assert_allclose((c1[0:3] + c2[0:3]) / 2, g[i, 0:3], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(c1[4:7], g[i, 4:7] + np.float32(-0.47000363), rtol=0, atol=1e-6)
    # past densify_until: unchanged
    out2, mk2, st2 = o.density_apply(g, acc, cnt, 15000, 1.0, 64.0, 64.0, 5.0, seed=4)
    assert np.array_equal(out2, g) and st2 == dict(num_pruned=0, num_cloned=0, num_split=0)
    # the MAX_GAUSSIANS cap drops clones first, then splits (density_control.mm:360-382)
    out3, mk3, st3 = o.density_apply(g, acc, cnt, 600, 1.0, 64.0, 64.0, 5.0, seed=4, max_gaussians=400)
    assert out3.shape[0] <= 400
