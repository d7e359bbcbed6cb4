"""Training loss: L1 + D-SSIM of MTLEngine::computeLoss
(mtl_engine.mm:769-853; shaders.metal:320-510).

CPU: the oracle against an independent numpy float32 restatement (same per-pixel operation and
summation order, window offsets dy-major) — bit-exact maps. GPU: the HIP kernel against the
oracle — bit-exact maps, mean within 1e-6 (both sum in fp64, in different orders)."""
from __future__ import annotations

import numpy as np
import pytest

from tests.kat_reference import expf as kat_expf

f32 = np.float32


def _images(w, h, seed, same=False):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (h, w, 4), dtype=np.uint32)
    a[..., 3] = 255
    b = a.copy() if same else np.clip(a.astype(np.int64) + rng.integers(-40, 41, (h, w, 4)), 0, 255).astype(np.uint32)
    b[..., 3] = 255
    pack = lambda x: (x[..., 0] | (x[..., 1] << 8) | (x[..., 2] << 16) | (x[..., 3] << 24)).astype(np.uint32)  # noqa: E731
    return pack(a), pack(b)


def _np_loss(r, g, lam):
    h, w = r.shape
    un = lambda v, c: ((v >> (8 * c)) & 0xFF).astype(np.float32) / f32(255.0)  # noqa: E731
    l1 = (np.abs(un(r, 0) - un(g, 0)) + np.abs(un(r, 1) - un(g, 1)) + np.abs(un(r, 2) - un(g, 2))) / f32(3.0)
    gx = (un(r, 0) + un(r, 1) + un(r, 2)) / f32(3.0)
    gy = (un(g, 0) + un(g, 1) + un(g, 2)) / f32(3.0)
    ys, xs = np.arange(h), np.arange(w)
    tss = f32(2.0) * f32(1.5) * f32(1.5)
    offs = [(dy, dx) for dy in range(-5, 6) for dx in range(-5, 6)]
    wts = [f32(kat_expf(f32(-f32(dx * dx + dy * dy)) / tss)) for dy, dx in offs]

    def shifted(img, dy, dx):
        return img[np.clip(ys + dy, 0, h - 1)][:, np.clip(xs + dx, 0, w - 1)]

    mx = np.zeros((h, w), np.float32)
    my = np.zeros((h, w), np.float32)
    ws = f32(0.0)
    for (dy, dx), wt in zip(offs, wts):
        ws = f32(ws + wt)
        mx = mx + wt * shifted(gx, dy, dx)
        my = my + wt * shifted(gy, dy, dx)
    mx = mx / ws
    my = my / ws
    vx = np.zeros((h, w), np.float32)
    vy = np.zeros((h, w), np.float32)
    cxy = np.zeros((h, w), np.float32)
    for (dy, dx), wt in zip(offs, wts):
        a = shifted(gx, dy, dx) - mx
        b = shifted(gy, dy, dx) - my
        vx = vx + wt * a * a
        vy = vy + wt * b * b
        cxy = cxy + wt * a * b
    vx, vy, cxy = vx / ws, vy / ws, cxy / ws
    C1, C2 = f32(0.01) * f32(0.01), f32(0.03) * f32(0.03)
    num = (f32(2.0) * mx * my + C1) * (f32(2.0) * cxy + C2)
    den = (mx * mx + my * my + C1) * (vx + vy + C2)
    dssim = np.minimum(np.maximum((f32(1.0) - num / den) / f32(2.0), f32(0.0)), f32(1.0))
    comb = (f32(1.0) - f32(lam)) * l1 + f32(lam) * dssim
    return np.stack([l1, dssim, comb]).astype(np.float32)


@pytest.mark.parametrize("w,h,same", [(40, 30, False), (7, 3, False), (1, 1, False), (33, 20, True)])
def test_oracle_loss_matches_numpy(w, h, same):
    from oracle import oracle
    r, g = _images(w, h, w * 131 + h, same)
    m, maps = oracle.loss(r, g, 0.2, threads=2)
    want = _np_loss(r, g, 0.2)
    assert np.array_equal(maps.view(np.uint32), want.view(np.uint32))
    assert abs(m - float(want[2].astype(np.float64).mean())) <= 1e-12
    if same:
        assert np.all(maps[0] == 0) and np.all(maps[1] == 0) and m == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,lam", [(1920, 1080, 0.2), (100, 75, 0.2), (17, 300, 0.5), (1, 1, 0.2)])
def test_gpu_loss_parity(dev, w, h, lam):
    import torch

    from gaussiansplatting_amd.rasterizer import Loss
    from oracle import oracle
    r, g = _images(w, h, 5 + w)
    m_ref, maps_ref = oracle.loss(r, g, lam)
    L = Loss()
    rt = torch.from_numpy(r.view(np.int32)).to(dev)
    gt = torch.from_numpy(g.view(np.int32)).to(dev)
    maps = torch.empty((3, h, w), dtype=torch.float32, device=dev)
    out = L.compute(rt, gt, lam, maps=maps)
    torch.cuda.synchronize()
    got = maps.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), maps_ref.view(np.uint32))
    assert abs(float(out.item()) - m_ref) <= 1e-6 * max(abs(m_ref), 1e-6)
