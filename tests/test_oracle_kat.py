"""Known-answer cross-check of the C oracle against an independent pure-Python restatement of the
reference kernels (tests/kat_reference.py) on small scenes (CPU only)."""
from __future__ import annotations

import numpy as np
import pytest

from gaussiansplatting_amd import scene
from tests import kat_reference as kat


def _oracle():
    from oracle import oracle
    return oracle


def _scene(n, w, h, seed, cam=None):
    g = scene.synthetic_gaussians(n, seed, w, h) if cam is None else \
        scene.synthetic_gaussians_camera(n, seed, w, h, **cam)
    rng = np.random.default_rng(seed)
    # sprinkle the awkward cases the reference handles specially
    g[0, 4:7] = [-4.0, 1.5, -4.0]      # anisotropy beyond 20:1 (projection rescales)
    g[1, 8:12] = 0.0                    # degenerate quaternion -> identity
    g[2, 12] = -7.0                     # opacity under the 0.005 pair filter
    g[3, 13] = 3.0                      # colour saturates (gradient zeroed)
    g[4, 0] = np.nan                    # NaN position -> culled
    g[5, 2] = 0.05                      # too close to the camera -> culled
    g[6, 4:7] = 2.5                     # big splat (many tiles)
    g[7:9] = g[9:11]                    # exact duplicates (equal depth keys)
    g[:, 12] += rng.normal(0, 0.1, n).astype(np.float32)
    return g


def test_exp_matches_python_restatement():
    o = _oracle()
    xs = np.linspace(-8.0, 8.0, 4001).astype(np.float32)
    for x in xs:
        assert np.float32(o.expf(float(x))) == kat.expf(x), x
    # accuracy of the pinned exp against the true exp
    e = np.array([o.expf(float(x)) for x in xs], np.float64)
    assert np.max(np.abs(e - np.exp(xs.astype(np.float64))) / np.exp(xs.astype(np.float64))) < 2e-7


def test_half_rounding_matches_numpy():
    o = _oracle()
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.normal(0, 1, 3000), rng.normal(0, 1e-5, 2000), rng.normal(0, 6e4, 500),
                           [6.1e-5, 5.96e-8, 2.98e-8, 65504.0, 65520.0, 1e-4, 0.99, 1 / 255]])
    for v in vals.astype(np.float32):
        with np.errstate(over="ignore"):
            want = np.float32(np.float16(v))
        got = np.float32(o.half(float(v)))
        assert (np.isnan(got) and np.isnan(want)) or got == want, v


@pytest.mark.parametrize("n,w,h,seed,general", [(24, 40, 36, 3, False), (40, 33, 47, 8, False),
                                                 (40, 48, 40, 5, True), (32, 37, 29, 6, True)])
def test_oracle_equals_python_restatement(n, w, h, seed, general):
    """general: a rotated, translated camera with fx != fy and an off-centre principal point
    (scene.general_camera): W in T = J W and W^T in the position gradient are not the identity."""
    o = _oracle()
    cam = scene.general_camera(w, h) if general else None
    g = _scene(n, w, h, seed, cam)
    u = scene.make_uniforms(w, h, **(cam or {}))
    gt = scene.synthetic_ground_truth(seed, 0, w, h)
    ref = kat.rasterize(g, u, w, h, gt)
    f = o.forward(g, u, w, h, threads=1)
    assert f.num_pairs == len(ref["keys"]) > 0
    assert np.array_equal(f.keys, ref["keys"])
    assert np.array_equal(f.values, ref["values"])
    assert np.array_equal(f.ranges, ref["ranges"])
    assert np.array_equal(f.last_idx, ref["last_idx"])
    assert np.array_equal(f.rgba8, ref["rgba8"])
    assert np.array_equal(f.rgb.view(np.uint32), ref["rgb"].view(np.uint32))
    proj = f.projected.view(scene.PROJECTED_DTYPE).reshape(-1)
    for i, p in enumerate(ref["projected"]):
        assert proj["radius"][i] == p["radius"], i
        assert tuple(proj["screen_pos"][i]) == p["screen"], i
        assert tuple(proj["conic"][i]) == p["conic"], i
        assert tuple(proj["cov2d"][i]) == p["cov"], i
        assert proj["opacity"][i] == p["opacity"], i
        assert tuple(proj["color"][i]) == p["color"], i
    gr, ab, nz = o.backward(g, f, f.rgba8, gt, threads=1)
    np.testing.assert_allclose(gr, ref["grad"], rtol=1e-12, atol=1e-30)
