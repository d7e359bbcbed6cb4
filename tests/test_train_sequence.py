"""Multi-iteration training-sequence parity (VERDICT r2 "next" 8): the reference's per-view
trainStep / train loop (mtl_engine.mm:856-1025, 1085-1192) driven through the library's Python
mirror for iterations 598..605, against the oracle after every stage of every iteration.

Per iteration: forward -> loss -> backward -> density accumulate -> Adam; densification when
500 < it < 15000 and it % 2 == 0 (apply, Adam moments follow the markers, accumulator reset:
:1108-1167); the opacity reset when it % 3 == 0 (raw opacity clamp, opacity and scale momentum
resets, accumulator reset: :1173-1192). The reference's own period is 100 / 3000 iterations; the
compressed schedule puts four applies and two resets into eight iterations.

Each stage is checked on identical inputs: the oracle's backward runs on the GPU's current
Gaussians, and the stages after it consume the GPU's gradients, so everything but the gradients
(within the §8c bar, tests/_helpers.compare_gradients) is compared bit for bit: the rendered image,
keys / values / ranges / lastIdx, the accumulators, the Gaussians and both Adam moments after every
step, the survivors of every apply, the opacity reset.

path = "records": the reference's data flow (gs_backward into GaussianGradients records, then
gs_density_accumulate and gs_adam_step). path = "fused": config 5's timed path, gs_backward_step
(the chain kernel feeding each Gaussian's gradient to the density statistics and to Adam in place,
with the cold SH moment lanes and the moments of never-reached Gaussians skipped -- gs_adam.hpp); the
GPU's gradients for the oracle's stages come from a gs_backward_packed of the same forward first
(the fused kernel's own gradients are bit-identical to it: test_backward_step_fused_equals_unfused),
so every fused step is also a second backward of one forward. Split children start with zero moments
(live flag 0) and turn live in the fused kernel when a pixel first reaches them."""
from __future__ import annotations

import numpy as np
import pytest

from gaussiansplatting_amd import scene
from tests._helpers import compare_forward, compare_gradients

pytestmark = pytest.mark.gpu

LRS = (0.00016, 0.005, 0.001, 0.025, 0.0025)  # trainStep's learning rates (mtl_engine.mm:1060-1069)


def _follow(m, v, markers):
    """Moments after an apply, walking the markers in the order density_control.mm:392-482 emits:
    kept -> its moments, clone -> the original's moments then a zeroed copy, split -> two zeroed
    children, pruned -> nothing (the library's gs_adam_follow_density)."""
    n_out = int(sum(0 if k == 1 else (1 if k == 0 else 2) for k in markers))
    em = np.zeros((n_out, 24), np.float32)
    ev = np.zeros((n_out, 24), np.float32)
    o = 0
    for i, k in enumerate(markers):
        if k == 1:
            continue
        if k in (0, 2):
            em[o], ev[o] = m[i], v[i]
        o += 1 if k == 0 else 2
    return em, ev


@pytest.mark.parametrize("path", ["records", "fused"])
@pytest.mark.parametrize("moments", ["follow", "reference"])
def test_train_iterations_598_to_605(dev, moments, path):
    """moments = "follow": after each apply the Adam moments follow the survivors (gs_adam_follow_density,
    the official 3DGS semantics); "reference": the reference's own sequence, resizeIfNeeded +
    resetStateForNewGaussians(oldCount) (mtl_engine.mm:1159-1166) -- the state is not permuted, only
    the tail past the old count is zeroed (gs_adam_resize + gs_adam_reset_new)."""
    import torch

    from gaussiansplatting_amd.rasterizer import (AdamOptimizer, DensityController, Loss, TiledRasterizer,
                                                  opacity_reset, unpack_gradients)
    from oracle import oracle as o
    w, h, n, seed = 320, 180, 20_000, 3
    f = float(w)
    extent = 1.1 * 0.25 * 3.5  # gs_train_headless: the 8-camera rig's spread
    g = scene.synthetic_gaussians(n, seed, w, h)
    u = scene.make_uniforms(w, h)
    gt = scene.synthetic_ground_truth(seed, 0, w, h)
    dgt = torch.from_numpy(gt.view(np.int32)).to(dev)
    dg = torch.from_numpy(g.copy()).to(dev)
    rast = TiledRasterizer(4 * n, 0, w, h)
    dc = DensityController(4 * n, 0)
    dc.set_scene_extent(extent)
    opt = AdamOptimizer(4 * n)
    loss = Loss()
    dc.reset_accumulator(n)
    # the oracle's state: Gaussians, Adam moments, density accumulators
    go = g.copy()
    st = o.AdamState(n)
    acc, cnt, pos = np.zeros(n, np.float32), np.zeros(n, np.uint32), np.zeros((n, 3), np.float32)
    applies = resets = 0
    zero_moments = None  # after an apply: the Gaussians whose moment records are all zero
    late_live = 0        # ... of which the next step gave non-zero moments (the live flag turned on)
    for it in range(598, 606):
        n = go.shape[0]
        assert dg.shape[0] == n
        assert np.array_equal(dg.cpu().numpy().view(np.uint32), go.view(np.uint32)), f"it {it}: Gaussians"
        # forward + loss
        img = torch.empty((h, w), dtype=torch.int32, device=dev)
        rgb = torch.empty((h, w, 3), dtype=torch.float32, device=dev)
        rast.forward(dg, u, img, rgb)
        lval = loss.compute(img, dgt)
        ref = o.forward(go, u, w, h)
        gpu = {"num_pairs": rast.num_pairs(), "rgba8": img.cpu().numpy().view(np.uint32), "rgb": rgb.cpu().numpy(),
               "ranges": rast.tile_ranges(), "last_idx": rast.last_idx(), "projected": rast.projected()}
        gpu["keys"], gpu["values"] = rast.sorted_pairs()
        compare_forward(gpu, ref)
        lref, _ = o.loss(ref.rgba8, gt)
        assert abs(float(lval.item()) - lref) <= 1e-5 * abs(lref), (float(lval.item()), lref)
        # backward
        grad = torch.empty((n, 28), dtype=torch.float32, device=dev)
        if path == "records":
            rast.backward(dg, grad, u, img, dgt)
        else:
            rows = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
            vs = torch.empty((n, 2), dtype=torch.float32, device=dev)
            rast.backward_rows(dg, rows, vs, u, img, dgt)
            unpack_gradients(rows, vs, grad)
        gg = grad.cpu().numpy()
        gr, ab, nz, sh, cd = o.backward_full(go, ref, ref.rgba8, gt)
        compare_gradients(gg, gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"iteration {it} ({path})")
        if path == "records":
            dc.accumulate_gradients(grad, n)
            opt.step(dg, grad, LRS)
        else:  # chain -> density statistics -> Adam per Gaussian, one kernel (the second backward of this forward)
            rast.backward_step(dg, u, img, dgt, opt, dc, LRS)
        # density accumulate (on the GPU's gradients)
        o.density_accumulate(gg, acc, cnt, pos)
        a2, c2, p2 = dc.read(n)
        assert np.array_equal(a2.view(np.uint32), acc.view(np.uint32)) and np.array_equal(c2, cnt)
        assert np.array_equal(p2.view(np.uint32), pos.view(np.uint32)), f"it {it}: accumulators"
        # Adam
        with np.errstate(invalid="ignore", over="ignore"):
            o.adam_step(go, gg, st, LRS)
        assert opt.timestep == st.t, (opt.timestep, st.t)
        m, v = opt.state(n)
        assert np.array_equal(dg.cpu().numpy().view(np.uint32), go.view(np.uint32)), f"it {it}: Adam step"
        assert np.array_equal(m.view(np.uint32), st.records("m").view(np.uint32)), f"it {it}: m"
        assert np.array_equal(v.view(np.uint32), st.records("v").view(np.uint32)), f"it {it}: v"
        if zero_moments is not None:
            late_live += int((zero_moments & (m != 0).any(axis=1)).sum())
            zero_moments = None
        # densification (mtl_engine.mm:1108-1167)
        if 500 < it < 15000 and it % 2 == 0:
            new, stats = dc.apply(dg, it, focal_length=f, image_width=f, avg_depth=6.0, seed=it)
            g2, markers, rst = o.density_apply(go, acc, cnt, it, extent, f, f, 6.0, it)
            assert stats == rst, (it, stats, rst)
            assert np.array_equal(new.cpu().numpy().view(np.uint32), g2.view(np.uint32)), f"it {it}: apply"
            n_out = g2.shape[0]
            if moments == "follow":
                opt.follow_density(dc, n, n_out)
                em, ev = _follow(*st_records(st), markers)
            else:
                opt.resize_if_needed(n_out)
                if n_out > n:
                    opt.reset_state_for_new_gaussians(n, n_out)
                m0, v0 = st_records(st)
                em = np.zeros((n_out, 24), np.float32)
                ev = np.zeros((n_out, 24), np.float32)
                keep = min(n, n_out)
                em[:keep], ev[:keep] = m0[:keep], v0[:keep]
            st.set_records(em, ev)
            m, v = opt.state(n_out)
            assert np.array_equal(m.view(np.uint32), em.view(np.uint32)), f"it {it}: m follow"
            assert np.array_equal(v.view(np.uint32), ev.view(np.uint32)), f"it {it}: v follow"
            dg, go = new.contiguous(), g2.copy()
            zero_moments = ~((em != 0).any(axis=1) | (ev != 0).any(axis=1))
            dc.reset_accumulator(n_out)
            acc, cnt, pos = np.zeros(n_out, np.float32), np.zeros(n_out, np.uint32), np.zeros((n_out, 3), np.float32)
            applies += 1
            assert rst["num_cloned"] + rst["num_split"] + rst["num_pruned"] > 0
        # opacity reset (mtl_engine.mm:1173-1192)
        if it % 3 == 0:
            nn = go.shape[0]
            opacity_reset(dg, -4.6)
            o.opacity_reset(go, -4.6)
            opt.reset_opacity_momentum(nn)
            opt.reset_scale_momentum(nn)
            em, ev = st_records(st)
            em[:, 3] = ev[:, 3] = 0.0
            em[:, 4:7] = ev[:, 4:7] = 0.0
            st.set_records(em, ev)
            m, v = opt.state(nn)
            assert np.array_equal(m.view(np.uint32), em.view(np.uint32)) and np.array_equal(v.view(np.uint32), ev.view(np.uint32))
            dc.reset_accumulator(nn)
            acc, cnt, pos = np.zeros(nn, np.float32), np.zeros(nn, np.uint32), np.zeros((nn, 3), np.float32)
            resets += 1
        torch.cuda.synchronize()
    assert applies == 4 and resets == 2
    assert late_live > 0  # Gaussians with zero moments after an apply (split children) stepped into life
    assert np.array_equal(dg.cpu().numpy().view(np.uint32), go.view(np.uint32))
    rast.close()
    dc.close()
    opt.close()


def st_records(st):
    return st.records("m"), st.records("v")
