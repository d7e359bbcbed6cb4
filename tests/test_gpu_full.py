"""Full-size GPU parity (SURVEY.md §8c at BASELINE.json's sizes), through the C-ABI.

  * config 2: the synthetic COLMAP scene (100k Gaussians initialised by gs_gaussians_from_colmap),
    1920x1080, views 0 and 7 — forward bit-exact, gradients within the bar;
  * config 4: the 1M scene under all 8 rig views — per view the forward bit-exact, then
    gs_backward_blend + a chunked gs_backward_chain into 56-B gradient rows + viewspace rows
    (bit-equal to one unchunked chain), both summed on the device over the views and compared,
    unpacked, with the oracle's sum over views;
  * config 5: 5M Gaussians (seed 5, view 0, ~69M pairs) — forward bit-exact on both tile-sort paths
    (one-pass counting sort, then the two-pass LSD sort the next frame picks at > 16M pairs),
    gradients within the bar, gs_density_apply at iteration 600 bit-exact against
    oracle.density_apply on the GPU's own accumulators, one Adam step bit-exact;
  * the N > 1 bench path: two ranks (gloo, both on GPU 0) through multiview.ViewStep (chunked chain
    + per-chunk all-reduce + unpack), against each rank's own single-view backward and the oracle.

The oracle runs on OMP_NUM_THREADS (or every core this process may use) threads; each test prints
progress lines (run with -s) and its gradient-bar audit."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from gaussiansplatting_amd import scene
from tests._helpers import compare_forward, compare_gradients, note, oracle_threads, run_gpu

pytestmark = pytest.mark.gpu

W, H = 1920, 1080


def _oracle():
    from oracle import oracle
    return oracle


def _chain(L, h, st, dg, n, ub, grad=None, packed=None, vs=None, a=0, b=None):
    from gaussiansplatting_amd import _lib
    b = n if b is None else b
    _lib.check(L.gs_backward_chain(h, st, dg.data_ptr(), grad.data_ptr() if grad is not None else None,
                                   packed.data_ptr() if packed is not None else None,
                                   vs.data_ptr() if vs is not None else None, n, ub, a, b - a),
               "gs_backward_chain")


@pytest.mark.timeout(900)
def test_config2_colmap_full_size(dev, tmp_path):
    from gaussiansplatting_amd import io
    c = scene.CONFIGS[2]
    io.synthetic_colmap(str(tmp_path), c["n"], c["seed"], W, H, views=8)
    sc = io.load_colmap(str(tmp_path))
    g = sc.gaussians()
    o, T = _oracle(), oracle_threads()
    assert g.shape[0] == c["n"]
    for view in (0, 7):
        u = sc.uniforms(view, W, H)
        gt = scene.synthetic_ground_truth(c["seed"], view, W, H)
        note(f"cfg2 view {view}: oracle forward ({T} threads)")
        ref = o.forward(g, u, W, H, max_pairs=16_000_000, threads=T)
        assert ref.num_pairs > 5_000_000
        gpu = run_gpu(g, u, W, H, gt=gt, reserve=16_000_000)
        assert gpu["rast"].frame_stats()["scan_errors"] == 0
        compare_forward(gpu, ref)
        note(f"cfg2 view {view}: {ref.num_pairs} pairs bit-exact; oracle backward")
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
        compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"cfg2 view {view}")
        gpu["rast"].close()
    sc.close()


@pytest.mark.timeout(900)
def test_general_camera_full_size(dev):
    """The bench size (1M Gaussians, 1920x1080) under scene.general_camera: a 15-degree rotation
    about a skew axis, a translation, fx != fy and an off-centre principal point, so W in T = J W
    (tiled_shaders.metal:218-225), W^T dL/dview (:556-565) and T^T dL/dcov2D T (:620-631) are all
    non-trivial. Forward bit-exact, gradients within the bar."""
    n, seed = 1_000_000, 33
    cam = scene.general_camera(W, H)
    g = scene.synthetic_gaussians_camera(n, seed, W, H, **cam)
    u = scene.make_uniforms(W, H, **cam)
    gt = scene.synthetic_ground_truth(seed, 0, W, H)
    o, T = _oracle(), oracle_threads()
    note(f"general camera: oracle forward ({T} threads)")
    ref = o.forward(g, u, W, H, max_pairs=16_000_000, threads=T)
    assert ref.num_pairs > 4_000_000
    gpu = run_gpu(g, u, W, H, gt=gt, reserve=16_000_000)
    assert gpu["rast"].frame_stats()["scan_errors"] == 0
    compare_forward(gpu, ref)
    note(f"general camera: {ref.num_pairs} pairs bit-exact; oracle backward")
    gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
    compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="general camera 1M 1080p")
    gpu["rast"].close()


@pytest.mark.timeout(900)
def test_colmap_rotated_poses_full_size(dev, tmp_path):
    """Config 2's size (100k COLMAP points, 1920x1080) with rotated image poses and a PINHOLE
    camera with fx != fy and an off-centre principal point (io.synthetic_colmap_posed), through
    gs_gaussians_from_colmap and gs_colmap_uniforms (mtl_engine.mm:637-682): views 0 and 5."""
    from gaussiansplatting_amd import io
    c = scene.CONFIGS[2]
    io.synthetic_colmap_posed(str(tmp_path), c["n"], c["seed"], W, H, views=8)
    sc = io.load_colmap(str(tmp_path))
    g = sc.gaussians()
    o, T = _oracle(), oracle_threads()
    for view in (0, 5):
        u = sc.uniforms(view, W, H)
        gt = scene.synthetic_ground_truth(c["seed"], view, W, H)
        ref = o.forward(g, u, W, H, max_pairs=16_000_000, threads=T)
        assert ref.num_pairs > 1_000_000
        gpu = run_gpu(g, u, W, H, gt=gt, reserve=16_000_000)
        compare_forward(gpu, ref)
        note(f"posed colmap view {view}: {ref.num_pairs} pairs bit-exact; oracle backward")
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
        compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"posed colmap view {view}")
        gpu["rast"].close()
    sc.close()


@pytest.mark.timeout(1200)
def test_config4_eight_views_packed_sum(dev):
    import torch

    from gaussiansplatting_amd import _lib
    from gaussiansplatting_amd.rasterizer import TiledRasterizer, _stream_ptr, _uniform_buffer
    c = scene.CONFIGS[4]
    n, seed = c["n"], c["seed"]
    g = scene.synthetic_gaussians(n, seed, W, H)
    o, T = _oracle(), oracle_threads()
    L = _lib.lib()
    r = TiledRasterizer(n, 0, W, H)
    r.reserve_pairs(16_000_000)
    dg = torch.from_numpy(g).to(dev)
    total = torch.zeros((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    vs_total = torch.zeros((n, 2), dtype=torch.float32, device=dev)
    pv = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    pu = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    vv = torch.empty((n, 2), dtype=torch.float32, device=dev)
    vu = torch.empty((n, 2), dtype=torch.float32, device=dev)
    ref_sum = np.zeros((n, 28))
    abs_sum = np.zeros((n, 28))
    noise_sum = np.zeros((n, 28))
    shadow_sum = np.zeros((n, 28))
    cond_sum = np.zeros((n, 28))
    cuts = [0, 7, 262_144, 333_333, 700_001, n]  # uneven chunks, one not a multiple of 64
    for view in range(c["views"]):
        u = scene.rig_uniforms(view, W, H)
        gt = scene.synthetic_ground_truth(seed, view, W, H)
        ref = o.forward(g, u, W, H, max_pairs=16_000_000, threads=T)
        gpu = run_gpu(g, u, W, H, rast=r, backward=False, dg=dg)
        compare_forward(gpu, ref)
        st, ub = _stream_ptr(None), _uniform_buffer(u)
        img = torch.from_numpy(gpu["rgba8"].view(np.int32)).to(dev)
        dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
        _lib.check(L.gs_backward_blend(r._h, st, dg.data_ptr(), n, ub, img.data_ptr(), dgt.data_ptr()), "blend")
        pv.fill_(float("nan"))
        vv.fill_(float("nan"))
        for a, b in zip(cuts, cuts[1:]):
            _chain(L, r._h, st, dg, n, ub, packed=pv, vs=vv, a=a, b=b)
        _chain(L, r._h, st, dg, n, ub, packed=pu, vs=vu)
        torch.cuda.synchronize()
        assert torch.equal(pv.view(torch.int32), pu.view(torch.int32)), f"view {view}: chunked chain != unchunked"
        assert torch.equal(vv.view(torch.int32), vu.view(torch.int32)), f"view {view}: chunked viewspace != unchunked"
        total += pv
        vs_total += vv
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
        ref_sum += gr
        abs_sum += ab
        noise_sum += nz
        shadow_sum += sh
        cond_sum += cd
        note(f"cfg4 view {view}: {ref.num_pairs} pairs, forward bit-exact, chunked chain == unchunked")
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev)
    _lib.check(L.gs_unpack_gradients(_stream_ptr(None), total.data_ptr(), vs_total.data_ptr(), grad.data_ptr(), n),
               "unpack")
    torch.cuda.synchronize()
    # the device sums 8 float32 views: 7 more roundings of <= 2^-24 |partial sum| each, far inside 1e-4
    compare_gradients(grad.cpu().numpy(), ref_sum, abs_sum, noise_sum, shadow_ref=shadow_sum,
                      cond_ref=cond_sum, label="cfg4 sum over 8 views")
    r.close()


@pytest.mark.timeout(1500)
def test_config5_five_million(dev):
    """Config 5 as bench_configs.py runs it: 5M Gaussians (rig view 0, ~23M pairs), backward, one
    density apply at iteration 600 (-> ~5.2M, the split Gaussians push the view to ~69M pairs),
    then the densified scene rendered twice, and two steps of bench_configs.py's timed path
    (gs_backward_step: the compacting chain feeding density statistics and Adam, cold SH lanes and
    never-reached Gaussians' moments skipped) bit-exact against the oracle's density_accumulate and
    adam_step on the GPU's gradients of the same forward."""
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer, DensityController, TiledRasterizer, unpack_gradients
    c = scene.CONFIGS[5]
    n, seed = c["n"], c["seed"]
    extent = 1.1 * 0.25 * 3.5  # bench_configs.py: the rig's camera spread
    o, T = _oracle(), oracle_threads()
    g = scene.synthetic_gaussians(n, seed, W, H)
    u = scene.rig_uniforms(0, W, H)
    gt = scene.synthetic_ground_truth(seed, 0, W, H)
    note(f"cfg5: oracle forward over {n} Gaussians ({T} threads)")
    ref = o.forward(g, u, W, H, max_pairs=80_000_000, threads=T)
    r = TiledRasterizer(2 * n, 0, W, H)
    r.reserve_pairs(80_000_000)
    dg = torch.from_numpy(g).to(dev)
    # frame 1: the one-pass counting sort (63488-pair scatter chunks), forced: with a reserve below
    # n * 256 the forward reads this frame's P back and the automatic choice would go to LSD
    r.set_tile_sort_path(1)
    gpu = run_gpu(g, u, W, H, gt=gt, rast=r, dg=dg)
    r.set_tile_sort_path(0)
    st = r.frame_stats()
    assert st["sort_passes_tile"] == 1 and st["scan_errors"] == 0
    compare_forward(gpu, ref)
    note(f"cfg5: {ref.num_pairs} pairs, one-pass tile sort bit-exact; oracle backward")
    gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
    compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"cfg5 5M ({ref.num_pairs} pairs)")
    del gr, ab, nz, ref
    grads = gpu["grad"]
    # density statistics of this view, then apply at iteration 600 (densify, no screen-size prune)
    dc = DensityController(n, 0)
    dc.set_scene_extent(extent)
    dc.reset_accumulator(n)
    dgrad = torch.from_numpy(grads).to(dev)
    dc.accumulate_gradients(dgrad)
    acc, cnt, pos = dc.read(n)
    acc_o = np.zeros(n, np.float32)
    cnt_o = np.zeros(n, np.uint32)
    pos_o = np.zeros((n, 3), np.float32)
    o.density_accumulate(grads, acc_o, cnt_o, pos_o)
    assert np.array_equal(acc.view(np.uint32), acc_o.view(np.uint32)) and np.array_equal(cnt, cnt_o)
    assert np.array_equal(pos.view(np.uint32), pos_o.view(np.uint32))
    new, dst = dc.apply(dg, 600, focal_length=float(W), image_width=float(W), avg_depth=5.0, seed=600)
    g2, _, rst = o.density_apply(g, acc, cnt, 600, extent, float(W), float(W), 5.0, 600)
    assert dst == rst, (dst, rst)
    assert rst["num_cloned"] + rst["num_split"] > 0
    assert np.array_equal(new.cpu().numpy().view(np.uint32), g2.view(np.uint32))
    note(f"cfg5: density apply at 600 bit-exact {rst} -> {g2.shape[0]} Gaussians")
    dc.close()
    # one Adam step on the GPU gradients (reference lrs, mtl_engine.mm:1060-1069)
    lrs = (0.00016, 0.005, 0.001, 0.025, 0.0025)
    opt = AdamOptimizer(n)
    opt.step(dg, dgrad, lrs)
    state = o.AdamState(n)
    go = g.copy()
    with np.errstate(invalid="ignore", over="ignore"):
        o.adam_step(go, grads, state, lrs)
    torch.cuda.synchronize()
    assert np.array_equal(dg.cpu().numpy().view(np.uint32), go.view(np.uint32))
    m, v = opt.state(n)
    assert np.array_equal(m.view(np.uint32), state.records("m").view(np.uint32))
    assert np.array_equal(v.view(np.uint32), state.records("v").view(np.uint32))
    note("cfg5: Adam step bit-exact")
    opt.close()
    del go, state, m, v, gpu, grads, dgrad, dg
    # bench_configs.py's timed state: the densified scene after 16 training steps through its timed
    # path (gs_backward_step) -- the split Gaussians grow and the view reaches ~69M pairs. The GPU
    # steps only produce the input; everything after is checked against the oracle on that input.
    dg2 = new.contiguous()
    n2 = dg2.shape[0]
    opt2 = AdamOptimizer(n2)
    img = torch.empty((H, W), dtype=torch.int32, device=dev)
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    for _ in range(16):
        r.forward(dg2, u, img)
        r.backward_step(dg2, u, img, dgt, opt2, None, lrs)
    torch.cuda.synchronize()
    g2 = dg2.cpu().numpy()
    note("cfg5: oracle forward of the densified scene after 16 steps")
    ref2 = o.forward(g2, u, W, H, max_pairs=80_000_000, threads=T)
    assert ref2.num_pairs > 60_000_000
    # automatic choice at P > 16M -> the two-pass LSD tile sort
    gpu2 = run_gpu(g2, u, W, H, gt=gt, rast=r, dg=dg2)
    st = r.frame_stats()
    assert st["sort_passes_tile"] == 2 and st["scan_errors"] == 0
    compare_forward(gpu2, ref2)
    note(f"cfg5: densified, {ref2.num_pairs} pairs, two-pass tile sort bit-exact; oracle backward")
    gr, ab, nz, sh, cd = o.backward_full(g2, ref2, ref2.rgba8, gt, threads=T)
    compare_gradients(gpu2["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"cfg5 densified ({ref2.num_pairs} pairs)")
    del gr, ab, nz
    # two steps of the timed path, continuing opt2's state (the oracle takes its moments and timestep)
    dc2 = DensityController(n2, 0)
    dc2.set_scene_extent(extent)
    dc2.reset_accumulator(n2)
    st2 = o.AdamState(n2)
    m0, v0 = opt2.state(n2)
    st2.set_records(m0, v0)
    st2.t = opt2.timestep
    del m0, v0
    go = g2.copy()
    acc_o, cnt_o, pos_o = np.zeros(n2, np.float32), np.zeros(n2, np.uint32), np.zeros((n2, 3), np.float32)
    rows = torch.empty((n2, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    vs = torch.empty((n2, 2), dtype=torch.float32, device=dev)
    gbuf = torch.empty((n2, 28), dtype=torch.float32, device=dev)
    for k in range(2):
        r.forward(dg2, u, img)
        r.backward_rows(dg2, rows, vs, u, img, dgt)
        unpack_gradients(rows, vs, gbuf)
        gg = gbuf.cpu().numpy()
        if k == 0:  # the oracle-checked gradients of this forward, through the 56-B rows
            rf = scene.ROW_FIELDS + scene.VIEWSPACE_FIELDS
            assert np.array_equal(gg[:, rf].view(np.uint32), gpu2["grad"][:, rf].view(np.uint32))
        r.backward_step(dg2, u, img, dgt, opt2, dc2, lrs)  # (the second backward of this forward)
        torch.cuda.synchronize()
        o.density_accumulate(gg, acc_o, cnt_o, pos_o)
        with np.errstate(invalid="ignore", over="ignore"):
            o.adam_step(go, gg, st2, lrs)
        assert opt2.timestep == st2.t
        assert np.array_equal(dg2.cpu().numpy().view(np.uint32), go.view(np.uint32)), f"cfg5 fused step {k}: Gaussians"
        m, v = opt2.state(n2)
        assert np.array_equal(m.view(np.uint32), st2.records("m").view(np.uint32)), f"cfg5 fused step {k}: m"
        assert np.array_equal(v.view(np.uint32), st2.records("v").view(np.uint32)), f"cfg5 fused step {k}: v"
        a2, c2, p2 = dc2.read(n2)
        assert np.array_equal(a2.view(np.uint32), acc_o.view(np.uint32)) and np.array_equal(c2, cnt_o)
        assert np.array_equal(p2.view(np.uint32), pos_o.view(np.uint32)), f"cfg5 fused step {k}: accumulators"
        del m, v, a2, c2, p2
    assert int(cnt_o.sum()) > 0
    note(f"cfg5: two fused training steps (gs_backward_step) bit-exact, {int((cnt_o > 0).sum())} Gaussians accumulated")
    opt2.close()
    dc2.close()
    del gpu2, rows, vs, gbuf, img, dgt, go, st2
    r.close()
    dg2.copy_(torch.from_numpy(g2).to(dev))  # (the fused steps moved it)
    # the one-pass sort at the same ~69M pairs
    r2 = TiledRasterizer(g2.shape[0], 0, W, H)
    r2.reserve_pairs(80_000_000)
    r2.set_tile_sort_path(1)
    gpu3 = run_gpu(g2, u, W, H, rast=r2, backward=False, dg=dg2)
    st = r2.frame_stats()
    assert st["sort_passes_tile"] == 1 and st["scan_errors"] == 0
    compare_forward(gpu3, ref2)
    note(f"cfg5: densified, one-pass tile sort at {ref2.num_pairs} pairs bit-exact")
    r2.close()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_hip_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    from gaussiansplatting_amd import multiview
    from gaussiansplatting_amd.rasterizer import DensityController, TiledRasterizer
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    c = scene.CONFIGS[4]
    n, seed = c["n"], c["seed"]
    g = scene.synthetic_gaussians(n, seed, W, H)
    u = scene.rig_uniforms(rank, W, H)  # rig camera = rank, as in bench.py
    gt = scene.synthetic_ground_truth(seed, rank, W, H)
    r = TiledRasterizer(n, 0, W, H)
    r.reserve_pairs(16_000_000)
    dg = torch.from_numpy(g).to(dev)
    out = torch.empty((H, W), dtype=torch.int32, device=dev)
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    own = torch.full((n, 28), float("nan"), dtype=torch.float32, device=dev)
    d_own = DensityController(0, 0)
    d_own.reset_accumulator(n)
    multiview.ViewStep(r, dg, u, out, dgt, own, world=1, density=d_own).step()
    torch.cuda.synchronize()
    for name, a in zip(("acc", "cnt", "pos"), d_own.read(n)):
        np.save(os.path.join(out_dir, f"own_{name}{rank}.npy"), a)
    np.save(os.path.join(out_dir, f"own{rank}.npy"), own.cpu().numpy())
    np.save(os.path.join(out_dir, f"img{rank}.npy"), out.cpu().numpy())
    grad = torch.full((n, 28), float("nan"), dtype=torch.float32, device=dev)
    packed = torch.full((n, scene.ROW_FLOATS), float("nan"), dtype=torch.float32, device=dev)
    d_step = DensityController(0, 0)
    d_step.reset_accumulator(n)
    step = multiview.ViewStep(r, dg, u, out, dgt, grad, packed, world=world, chunks=4, density=d_step)
    step.compute()
    step.finish()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, f"sum{rank}.npy"), grad.cpu().numpy())
    for name, a in zip(("acc", "cnt", "pos"), d_step.read(n)):
        np.save(os.path.join(out_dir, f"step_{name}{rank}.npy"), a)
    d_own.close()
    d_step.close()
    dist.barrier()
    dist.destroy_process_group()
    r.close()


@pytest.mark.timeout(900)
def test_two_rank_gloo_hip_view_step(dev, tmp_path):
    """The bench's N > 1 step (multiview.ViewStep: gs_backward_blend, then per chunk the chain into
    gradient rows + that chunk's async all-reduce + unpack), two ranks on GPU 0 over gloo: both
    replicas' summed fields bit-identical, equal to the float32 sum of the two ranks' own single-view
    gradients bit for bit, each rank's viewspace its own view's, each rank's density statistics its
    own view's (pos_accum not summed over ranks), and within the bar of the oracle's sum over the
    two views."""
    import torch.multiprocessing as mp
    port = _free_port()
    note("2-rank gloo: spawning")
    mp.spawn(_gloo_hip_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    s0, s1 = np.load(tmp_path / "sum0.npy"), np.load(tmp_path / "sum1.npy")
    rf, vf = scene.ROW_FIELDS, scene.VIEWSPACE_FIELDS
    assert np.array_equal(s0[:, rf].view(np.uint32), s1[:, rf].view(np.uint32)), "replicas differ"
    own = [np.load(tmp_path / f"own{r}.npy") for r in range(2)]
    assert np.array_equal(s0[:, rf].view(np.uint32), (own[0] + own[1])[:, rf].view(np.uint32))
    # the screen-space gradient is per rank (density statistics per view), never reduced
    for r, sr in enumerate((s0, s1)):
        assert np.array_equal(sr[:, vf].view(np.uint32), own[r][:, vf].view(np.uint32))
    # density statistics on the N > 1 path: each rank's own view (accumulated per chunk before the
    # chunk's reduce), bit-equal to accumulating its own single-view records; pos_accum is not the
    # sum over ranks
    for r in range(2):
        for name in ("acc", "cnt", "pos"):
            a, b = np.load(tmp_path / f"step_{name}{r}.npy"), np.load(tmp_path / f"own_{name}{r}.npy")
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (r, name)
        assert np.load(tmp_path / f"own_cnt{r}.npy").sum() > 0
    s0 = s0.copy()
    s0[:, vf] = own[0][:, vf] + own[1][:, vf]
    c = scene.CONFIGS[4]
    g = scene.synthetic_gaussians(c["n"], c["seed"], W, H)
    o, T = _oracle(), oracle_threads()
    ref_sum = abs_sum = noise_sum = shadow_sum = cond_sum = 0.0
    for view in range(2):
        u = scene.rig_uniforms(view, W, H)
        gt = scene.synthetic_ground_truth(c["seed"], view, W, H)
        ref = o.forward(g, u, W, H, max_pairs=16_000_000, threads=T)
        assert np.array_equal(np.load(tmp_path / f"img{view}.npy").view(np.uint32), ref.rgba8)
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=T)
        ref_sum, abs_sum, noise_sum = ref_sum + gr, abs_sum + ab, noise_sum + nz
        shadow_sum, cond_sum = shadow_sum + sh, cond_sum + cd
    compare_gradients(s0, ref_sum, abs_sum, noise_sum, shadow_ref=shadow_sum, cond_ref=cond_sum,
                      label="2-rank gloo sum of views 0+1")
