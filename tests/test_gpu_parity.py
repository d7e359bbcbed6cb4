"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical inputs."""
from __future__ import annotations

import numpy as np
import pytest

from gaussiansplatting_amd import scene
from tests._helpers import compare_forward, compare_gradients, oracle_threads, run_gpu

pytestmark = pytest.mark.gpu


def _oracle():
    from oracle import oracle
    return oracle


def _case(n, w, h, seed, view=0):
    g = scene.synthetic_gaussians(n, seed, w, h)
    u = scene.make_uniforms(w, h)
    gt = scene.synthetic_ground_truth(seed, view, w, h)
    return g, u, gt


def _full(g, u, gt, w, h, **kw):
    o = _oracle()
    ref = o.forward(g, u, w, h)
    gpu = run_gpu(g, u, w, h, gt=gt, **kw)
    compare_forward(gpu, ref)
    if ref.num_pairs > 0:
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt)
        compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=kw.pop("label", ""))
    return gpu, ref


def test_config1_parity(dev):
    c = scene.CONFIGS[1]
    g, u, gt = _case(c["n"], c["width"], c["height"], c["seed"])
    gpu, ref = _full(g, u, gt, c["width"], c["height"])
    assert ref.num_pairs > 10_000
    st = gpu["rast"].frame_stats()
    assert st["sort_passes_tile"] == 1  # one-pass counting sort
    assert st["scan_errors"] == 0  # no cross-workgroup scan gave up waiting
    # reference self-checks (tiled_rasterizer.mm:577-636): coverage == P, contiguous ranges
    assert int(gpu["ranges"][:, 1].sum()) == gpu["num_pairs"]


def test_bench_workload_parity(dev):
    """The bench workload itself (configs[2]/[3]: 1M Gaussians, 1920x1080, rig view 0, 4.65M
    pairs): forward bit-exact, gradients within the section-4 tolerance, against the oracle."""
    c = scene.CONFIGS[3]
    w, h, seed = c["width"], c["height"], c["seed"]
    g = scene.synthetic_gaussians(c["n"], seed, w, h)
    u = scene.rig_uniforms(0, w, h)
    gt = scene.synthetic_ground_truth(seed, 0, w, h)
    o = _oracle()
    ref = o.forward(g, u, w, h, max_pairs=16_000_000, threads=oracle_threads())
    assert ref.num_pairs > 4_000_000
    gpu = run_gpu(g, u, w, h, gt=gt, reserve=16_000_000)
    assert gpu["rast"].frame_stats()["scan_errors"] == 0
    compare_forward(gpu, ref)
    gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt, threads=oracle_threads())
    audit = compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="bench workload (cfg3, rig view 0)")
    # the widened entries belong to a handful of Gaussians (r03: reached only deep in long lists),
    # 27-32 entries measured: an entry-count cap near that level, so a precision regression of the
    # backward shows here before it reaches the 1e-5 budget (~160 entries)
    assert audit["widened_gaussians"] <= 8, audit
    assert audit["widened_budgeted"] <= 40, audit


def test_backward_split_bit_identical(dev):
    """The backward list split (gs_set_backward_split): off, the 100 heaviest tiles, and every tile
    (the default) give bit-identical gradients -- every list entry is processed by one wave with the
    same per-pixel operations in the same order, the front half continuing from the back half's
    handed-over state -- and within the bar of the oracle; two scenes on one handle (the handover
    words carry the frame tag)."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h = 320, 180
    o = _oracle()
    rs = {s: TiledRasterizer(30_000, 0, w, h) for s in (0, 100, -1)}
    for s, r in rs.items():
        r.set_backward_split(s)
    for n, seed in [(30_000, 51), (9_000, 52)]:
        g, u, gt = _case(n, w, h, seed)
        ref = o.forward(g, u, w, h)
        out = {}
        for s, r in rs.items():
            gpu = run_gpu(g, u, w, h, gt=gt, rast=r)
            compare_forward(gpu, ref)
            assert r.frame_stats()["scan_errors"] == 0
            out[s] = gpu["grad"]
        assert np.array_equal(out[0].view(np.uint32), out[100].view(np.uint32))
        assert np.array_equal(out[0].view(np.uint32), out[-1].view(np.uint32))
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt)
        compare_gradients(out[-1], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"split n={n}")
    for r in rs.values():
        r.close()


def test_chain_kernels_bit_identical(dev):
    """The plain and the compacting chain kernel (gs_set_chain_compact 0 / 1) give bit-identical
    gradients, on a scene whose Gaussians are mostly reached and on a deep one where most are not
    (pixels saturated long before the lists end), and the automatic choice matches both."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h = 256, 192
    o = _oracle()
    for n, seed, boost in [(20_000, 71, 0.0), (60_000, 72, 1.5)]:
        g, u, gt = _case(n, w, h, seed)
        if boost:
            g[:, 4:7] += boost  # large splats: deep lists, most Gaussians behind saturated pixels
        out = {}
        for mode in (0, 1, -1):
            r = TiledRasterizer(n, 0, w, h)
            r.set_chain_compact(mode)
            out[mode] = run_gpu(g, u, w, h, gt=gt, rast=r)["grad"]
            r.close()
        assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32)), n
        assert np.array_equal(out[0].view(np.uint32), out[-1].view(np.uint32)), n
    ref = o.forward(g, u, w, h)
    gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt)
    compare_gradients(out[1], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="compacting chain, deep lists")


def test_packed_backward_matches(dev):
    """gs_backward_packed (gradient rows + viewspace rows) + gs_unpack_gradients (the multi-GPU path)
    == gs_backward, bit for bit; gs_density_accumulate_rows and gs_adam_step_rows on the rows ==
    gs_density_accumulate and gs_adam_step on the records, bit for bit (config 5's path)."""
    import torch
    from gaussiansplatting_amd import _lib
    from gaussiansplatting_amd.rasterizer import (AdamOptimizer, DensityController, _stream_ptr,
                                                  _uniform_buffer, unpack_gradients)
    w, h = 320, 180
    g, u, gt = _case(20_000, w, h, 9)
    gpu = run_gpu(g, u, w, h, gt=gt)
    r = gpu["rast"]
    n = g.shape[0]
    dg = torch.from_numpy(g).to(dev)
    img = torch.from_numpy(gpu["rgba8"].view(np.int32)).to(dev)
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    rows = torch.full((n, scene.ROW_FLOATS), 3.0, dtype=torch.float32, device=dev)
    vs = torch.full((n, 2), 4.0, dtype=torch.float32, device=dev)
    grad = torch.full((n, 28), 5.0, dtype=torch.float32, device=dev)
    L = _lib.lib()
    _lib.check(L.gs_backward_packed(r._h, _stream_ptr(None), dg.data_ptr(), rows.data_ptr(), vs.data_ptr(), n,
                                    _uniform_buffer(u), img.data_ptr(), dgt.data_ptr()), "packed")
    unpack_gradients(rows, vs, grad)
    torch.cuda.synchronize()
    ref = gpu["grad"]
    assert np.array_equal(grad.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(rows.cpu().numpy().view(np.uint32), ref[:, scene.ROW_FIELDS].view(np.uint32))
    # without viewspace rows: the same gradient rows
    rows2 = torch.full((n, scene.ROW_FLOATS), 3.0, dtype=torch.float32, device=dev)
    r.backward_rows(dg, rows2, None, u, img, dgt)
    torch.cuda.synchronize()
    assert torch.equal(rows.view(torch.int32), rows2.view(torch.int32))
    # density statistics and Adam from rows == from records (two steps, moments included)
    drec = torch.from_numpy(ref).to(dev)
    dens_a, dens_b = DensityController(n, 0), DensityController(n, 0)
    dens_a.reset_accumulator(n)
    dens_b.reset_accumulator(n)
    for _ in range(2):
        dens_a.accumulate_gradients(drec, n)
        dens_b.accumulate_rows(rows, vs, n)
    for x, y in zip(dens_a.read(n), dens_b.read(n)):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))
    ga, gb = dg.clone(), dg.clone()
    ad_a, ad_b = AdamOptimizer(n, 0), AdamOptimizer(n, 0)
    for _ in range(2):
        ad_a.step(ga, drec)
        ad_b.step_rows(gb, rows)
    torch.cuda.synchronize()
    assert torch.equal(ga.view(torch.int32), gb.view(torch.int32))
    for x, y in zip(ad_a.state(n), ad_b.state(n)):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    # a shard: rows of Gaussians [first, first + count) only
    gc = dg.clone()
    ad_c = AdamOptimizer(n, 0)
    first, count = 5000, 7001
    ad_c.step_rows(gc, rows[first:first + count].contiguous(), first=first, count=count)
    ad_d = AdamOptimizer(n, 0)
    gd = dg.clone()
    ad_d.step(gd, drec)
    torch.cuda.synchronize()
    assert torch.equal(gc[first:first + count].view(torch.int32), gd[first:first + count].view(torch.int32))
    assert torch.equal(gc[:first].view(torch.int32), dg[:first].view(torch.int32))
    assert torch.equal(gc[first + count:].view(torch.int32), dg[first + count:].view(torch.int32))


def test_split_backward_matches(dev):
    """gs_backward_blend + gs_backward_chain over uneven chunks (packed and record outputs) ==
    gs_backward, bit for bit; range and state errors are reported."""
    import torch
    from gaussiansplatting_amd import _lib
    from gaussiansplatting_amd.rasterizer import _stream_ptr, _uniform_buffer
    w, h = 320, 180
    g, u, gt = _case(20_000, w, h, 9)
    gpu = run_gpu(g, u, w, h, gt=gt)
    r = gpu["rast"]
    n = g.shape[0]
    dg = torch.from_numpy(g).to(dev)
    img = torch.from_numpy(gpu["rgba8"].view(np.int32)).to(dev)
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    L, st, ub = _lib.lib(), _stream_ptr(None), _uniform_buffer(u)
    packed = torch.full((n, scene.ROW_FLOATS), 3.0, dtype=torch.float32, device=dev)
    vs = torch.full((n, 2), 4.0, dtype=torch.float32, device=dev)
    grad = torch.full((n, 28), 5.0, dtype=torch.float32, device=dev)
    _lib.check(L.gs_backward_blend(r._h, st, dg.data_ptr(), n, ub, img.data_ptr(), dgt.data_ptr()), "blend")
    for a, b in [(0, 7), (7, 5000), (5000, 12345), (12345, n)]:
        _lib.check(L.gs_backward_chain(r._h, st, dg.data_ptr(), None, packed.data_ptr(), vs.data_ptr(), n, ub, a,
                                       b - a), "chain")
        _lib.check(L.gs_backward_chain(r._h, st, dg.data_ptr(), grad.data_ptr(), None, None, n, ub, a, b - a), "chain")
    full = torch.empty((n, 28), dtype=torch.float32, device=dev)
    _lib.check(L.gs_unpack_gradients(st, packed.data_ptr(), vs.data_ptr(), full.data_ptr(), n), "unpack")
    torch.cuda.synchronize()
    assert np.array_equal(grad.cpu().numpy().view(np.uint32), gpu["grad"].view(np.uint32))
    assert np.array_equal(full.cpu().numpy().view(np.uint32), gpu["grad"].view(np.uint32))
    assert L.gs_backward_chain(r._h, st, dg.data_ptr(), grad.data_ptr(), None, None, n, ub, n - 1, 2) != 0
    assert L.gs_backward_chain(r._h, st, dg.data_ptr(), grad.data_ptr(), packed.data_ptr(), None, n, ub, 0, 1) != 0
    assert L.gs_backward_chain(r._h, st, dg.data_ptr(), grad.data_ptr(), None, vs.data_ptr(), n, ub, 0, 1) != 0


@pytest.mark.parametrize("w,h", [(100, 75), (17, 300), (256, 1)])
def test_ragged_images(dev, w, h):
    g, u, gt = _case(3000, w, h, 11)
    _full(g, u, gt, w, h)


def test_many_tiles_two_pass_sort(dev):
    """Over kTileSortMaxTiles (12288) tiles the pairs take the two-pass LSD tile sort instead of
    the one-pass counting sort; both must give the reference's order."""
    w, h = 2064, 1620  # 129 x 102 = 13158 tiles
    g, u, gt = _case(20_000, w, h, 23)
    gpu, ref = _full(g, u, gt, w, h)
    assert gpu["rast"].frame_stats()["sort_passes_tile"] == 2


def test_wide_tile_ids_three_pass_sort(dev):
    """Over 65536 tiles the tile ids no longer fit 16 bits: the emission writes u32 keys and the LSD
    tile sort runs three passes on u32 keys with the binary-search ranges (up to 65536 tiles: u16
    keys, and the last pass builds the ranges itself)."""
    w, h = 4400, 4200  # 275 x 263 = 72325 tiles, 17 tile bits
    g, u, gt = _case(20_000, w, h, 29)
    gpu, ref = _full(g, u, gt, w, h)
    st = gpu["rast"].frame_stats()
    assert st["sort_passes_tile"] == 3 and st["tile_sort_path"] == 2 and st["scan_errors"] == 0


@pytest.mark.parametrize("path", [1, 2])
@pytest.mark.parametrize("w,h,n", [(256, 256, 10_000), (1920, 1080, 100_000), (333, 77, 5_000)])
def test_tile_sort_paths(dev, path, w, h, n):
    """Both tile-sort implementations (gs_set_tile_sort_path: 1 one-pass counting sort, 2 8-bit LSD
    passes) give the reference's sorted pairs and ranges, and the whole forward bit-exact; twice on
    one handle (the one-pass sort's fan-in words are re-armed per frame)."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    g, u, gt = _case(n, w, h, 60 + path)
    ref = _oracle().forward(g, u, w, h)
    r = TiledRasterizer(n, 0, w, h)
    r.set_tile_sort_path(path)
    for _ in range(2):
        gpu = run_gpu(g, u, w, h, gt=gt, rast=r, backward=False)
        compare_forward(gpu, ref)
        st = r.frame_stats()
        assert st["scan_errors"] == 0
        tb = max(1, (scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1] - 1).bit_length())
        assert st["sort_passes_tile"] == (1 if path == 1 else (tb + 7) // 8)
        assert st["tile_sort_path"] == path
    r.close()


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("path", [1, 2])
@pytest.mark.parametrize("w,h,n,zlevels", [(256, 256, 10_000, 0), (64, 48, 60_000, 0), (1920, 1080, 100_000, 0),
                                             (256, 192, 30_000, 3), (64, 48, 60_000, 5), (320, 240, 40_000, -1),
                                             (128, 128, 40_000, 0)])
def test_depth_sort_modes(dev, mode, path, w, h, n, zlevels):
    """Both depth orders (gs_set_depth_sort: 1 the global sort of the N depth keys before a
    depth-order emission, 2 Gaussian-order emission then every tile list sorted by depth on its own)
    under both tile sorts give the reference's sorted pairs, ranges and the whole forward bit-exact.
    The 64x48 scenes put ~4k-60k pairs into each of the 12 tiles (the per-tile sort's chunked path,
    many chunks), the 128x128 one ~1k-3k into each of 64 (the workgroup bucket sort); zlevels > 0 quantises the Gaussians' depths to a few values, so most depth keys tie
    and the order among them is the Gaussian order (the stability of both sorts); zlevels = -1 spreads
    the depths over [0.3, 40] (keys 26 bits apart: the one-wave sort works on key - min key)."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    g, u, gt = _case(n, w, h, 70 + zlevels + (n % 13))
    if zlevels < 0:
        z0 = g[:, 2].copy()
        znew = np.exp(np.random.default_rng(5).uniform(np.log(0.3), np.log(40.0), n)).astype(np.float32)
        g[:, 0] *= znew / z0  # keep the splats on screen
        g[:, 1] *= znew / z0
        g[:, 2] = znew
        g[:, 4:7] += np.log(znew / z0)[:, None]  # and at their pixel size
    elif zlevels:
        z = g[:, 2].copy()
        lv = np.linspace(z.min(), z.max(), zlevels)
        g[:, 2] = lv[np.argmin(np.abs(z[:, None] - lv[None, :]), axis=1)]
    ref = _oracle().forward(g, u, w, h, max_pairs=16_000_000, threads=oracle_threads())
    tiles = scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]
    # the per-tile order on the one-pass path also runs with the pair buffers at the worst case, where
    # no offset scan runs (the tile sort's walks number the slots and write goff and P themselves)
    for reserve in [None] + ([n * min(256, tiles)] if mode == 2 and path == 1 else []):
        r = TiledRasterizer(n, 0, w, h)
        if reserve:
            r.reserve_pairs(reserve)
        r.set_tile_sort_path(path)
        r.set_depth_sort(mode)
        for _ in range(2):
            gpu = run_gpu(g, u, w, h, gt=gt, rast=r, backward=False)
            compare_forward(gpu, ref)
            st = r.frame_stats()
            assert st["scan_errors"] == 0 and st["tile_sort_path"] == path
            assert st["sort_passes_depth"] == (4 if mode == 1 else 0)
            assert r.num_pairs() == ref.keys.size
        r.close()
    if zlevels > 0:
        keys = ref.keys.astype(np.uint64)
        assert np.unique(keys).size < keys.size // 4  # mostly ties


def test_own_offsets_match_offset_scan(dev):
    """The per-tile order with the pair buffers at the worst case numbers the slots inside the tile
    sort's walks (no offset scan; its scatter writes goff, the raster records' slot field and P):
    forward outputs, gradients, the projected records and the frame stats are bit-identical to the
    same frames with the offset scan (default reservation), over two frames (the frame tag turns)."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h, n = 320, 240, 40_000
    g, u, gt = _case(n, w, h, 77)
    g[::7, scene.G_OPACITY] = -9.0  # near-transparent Gaussians between the live ones (raw opacity)
    tiles = scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]
    runs = []
    for reserve in (None, n * min(256, tiles)):
        r = TiledRasterizer(n, 0, w, h)
        if reserve:
            r.reserve_pairs(reserve)
        r.set_depth_sort(2)
        frames = [run_gpu(g, u, w, h, gt=gt, rast=r) for _ in range(2)]
        runs.append((frames, r.frame_stats()))
        r.close()
    (fa, sa), (fb, sb) = runs
    for a, b in zip(fa, fb):
        for k in ("rgba8", "keys", "values", "ranges", "last_idx"):
            assert np.array_equal(a[k], b[k]), k
        assert np.array_equal(a["rgb"].view(np.uint32), b["rgb"].view(np.uint32))
        assert np.array_equal(a["grad"].view(np.uint32), b["grad"].view(np.uint32)), "gradients differ"
        assert np.array_equal(a["projected"].view(np.uint32), b["projected"].view(np.uint32))
        assert a["num_pairs"] == b["num_pairs"]
    assert sa["sort_passes_depth"] == sb["sort_passes_depth"] == 0 and sa["scan_errors"] == sb["scan_errors"] == 0
    # everything culled: P = 0 from the scatter's own count, the forward's early return (no render,
    # lastIdx = UINT_MAX, tiled_rasterizer.mm:463-467), then a live frame on the same handle
    r = TiledRasterizer(n, 0, w, h)
    r.reserve_pairs(n * min(256, tiles))
    r.set_depth_sort(2)
    dead = g.copy()
    dead[:, scene.G_OPACITY] = -30.0
    z = run_gpu(dead, u, w, h, rast=r, backward=False)
    assert z["num_pairs"] == 0 and np.all(z["last_idx"] == 0xFFFFFFFF)
    live = run_gpu(g, u, w, h, gt=gt, rast=r)
    assert np.array_equal(live["values"], fa[0]["values"]) and np.array_equal(live["rgba8"], fa[0]["rgba8"])
    assert np.array_equal(live["grad"].view(np.uint32), fa[0]["grad"].view(np.uint32))
    r.close()


def test_large_pair_count_sort(dev):
    """~25M pairs: the one-pass tile sort's slices exceed one scatter chunk (63488 pairs), so the
    chunked path (counters re-armed per chunk, base advanced per chunk) is exercised. Checked
    against the oracle's project -> generateTilePairs -> 64-bit sort -> buildTileRanges."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    import torch
    w, h = 1920, 1080
    g = scene.synthetic_gaussians(250_000, 41, w, h)
    g[:, 4:7] += 2.3  # large splats: ~100 tiles each
    u = scene.make_uniforms(w, h)
    keys, vals, ranges = _oracle().sorted_pairs(g, u, w, h)
    assert keys.size > 256 * 63488
    r = TiledRasterizer(g.shape[0], 0, w, h)
    r.reserve_pairs(g.shape[0] * 256)  # worst case: no P readback, so frame 1 takes the one-pass sort
    out = torch.empty((h, w), dtype=torch.int32, device="cuda:0")
    r.forward(torch.from_numpy(g).to("cuda:0"), u, out)
    torch.cuda.synchronize()
    assert r.num_pairs() == keys.size
    gk, gv = r.sorted_pairs()
    assert np.array_equal(gk, keys)
    assert np.array_equal(gv, vals)
    gr = r.tile_ranges()
    assert np.array_equal(gr, ranges)
    assert r.frame_stats()["sort_passes_tile"] == 1
    # the next frame sees the previous P (> 16M) and takes the two-pass LSD path: same result
    r.forward(torch.from_numpy(g).to("cuda:0"), u, out)
    torch.cuda.synchronize()
    assert r.frame_stats()["sort_passes_tile"] == 2
    gk2, gv2 = r.sorted_pairs()
    assert np.array_equal(gk2, keys) and np.array_equal(gv2, vals)
    assert np.array_equal(r.tile_ranges(), ranges)
    # and the classic 8-bit LSD passes
    r.set_tile_sort_path(2)
    r.forward(torch.from_numpy(g).to("cuda:0"), u, out)
    torch.cuda.synchronize()
    gk3, gv3 = r.sorted_pairs()
    assert np.array_equal(gk3, keys) and np.array_equal(gv3, vals)
    assert np.array_equal(r.tile_ranges(), ranges)
    assert r.frame_stats()["scan_errors"] == 0
    r.close()


def _os_items(n):
    """gs_sort.hip os_items: keys per thread of the depth sort's partitions for n keys."""
    if n <= 1 << 21:
        return 4
    cost = {it: -(-(-(-n // (1024 * it))) // 256) * it for it in (8, 10, 12)}
    return min(cost, key=lambda it: (cost[it], it))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,zlevels", [(2_300_000, 0), (3_000_000, 7), (6_000_000, 0)])
def test_depth_sort_partition_sizes(dev, n, zlevels):
    """The global depth sort picks its partition size from n (10, 12 and 8 keys per thread here:
    gs_sort.hip os_items); each size gives the reference's sorted pairs and tile ranges bit-exact,
    over two frames (the partition tickets and status words re-armed). zlevels > 0 quantises the
    depths so most keys tie (the sort's stability across partitions)."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    import torch
    assert [_os_items(m) for m in (100_000, 2_300_000, 3_000_000, 5_200_000, 6_000_000)] == [4, 10, 12, 10, 8]
    w, h = 1920, 1080
    g = scene.synthetic_gaussians(n, 43 + zlevels, w, h)
    g[:, 4:7] -= 0.7  # small splats: a few tiles each
    if zlevels:
        z = g[:, 2].copy()
        lv = np.linspace(z.min(), z.max(), zlevels)
        g[:, 2] = lv[np.argmin(np.abs(z[:, None] - lv[None, :]), axis=1)]
    u = scene.make_uniforms(w, h)
    keys, vals, ranges = _oracle().sorted_pairs(g, u, w, h)
    r = TiledRasterizer(n, 0, w, h)
    r.set_depth_sort(1)
    out = torch.empty((h, w), dtype=torch.int32, device="cuda:0")
    gd = torch.from_numpy(g).to("cuda:0")
    for _ in range(2):
        r.forward(gd, u, out)
        torch.cuda.synchronize()
        st = r.frame_stats()
        assert st["sort_passes_depth"] == 4 and st["scan_errors"] == 0
        assert r.num_pairs() == keys.size
        gk, gv = r.sorted_pairs()
        assert np.array_equal(gk, keys) and np.array_equal(gv, vals)
        assert np.array_equal(r.tile_ranges(), ranges)
    r.close()


def test_rig_camera_views(dev):
    w, h = 320, 180
    g = scene.synthetic_gaussians(20_000, 4, w, h)
    for j in (0, 3, 7):
        u = scene.rig_uniforms(j, w, h)
        gt = scene.synthetic_ground_truth(4, j, w, h)
        _full(g, u, gt, w, h)


def test_general_camera(dev):
    """A rotated, translated camera with fx != fy and an off-centre principal point
    (scene.general_camera): the view rotation enters T = J W (tiled_shaders.metal:218-225), the
    world-position gradient W^T dL/dview (:556-565) and T^T dL/dcov2D T (:620-631)."""
    w, h = 320, 180
    cam = scene.general_camera(w, h)
    g = scene.synthetic_gaussians_camera(20_000, 44, w, h, **cam)
    u = scene.make_uniforms(w, h, **cam)
    gt = scene.synthetic_ground_truth(44, 0, w, h)
    gpu, ref = _full(g, u, gt, w, h)
    assert ref.num_pairs > 50_000


def test_colmap_rotated_poses(dev, tmp_path):
    """A COLMAP scene whose images carry rotated poses (io.synthetic_colmap_posed), initialised by
    gs_gaussians_from_colmap, rendered through gs_colmap_uniforms from three of its views."""
    from gaussiansplatting_amd import io
    w, h = 480, 270
    io.synthetic_colmap_posed(str(tmp_path), 20_000, 45, w, h)
    sc = io.load_colmap(str(tmp_path))
    g = sc.gaussians()
    for view in (0, 3, 6):
        u = sc.uniforms(view, w, h)
        gt = scene.synthetic_ground_truth(45, view, w, h)
        _full(g, u, gt, w, h)
    sc.close()


def test_empty_and_culled(dev):
    w, h = 64, 48
    u = scene.make_uniforms(w, h)
    # n = 0
    gpu = run_gpu(np.zeros((0, 28), np.float32), u, w, h, backward=False)
    assert gpu["num_pairs"] == 0
    assert np.all(gpu["last_idx"] == 0xFFFFFFFF)
    assert np.all(gpu["rgba8"] == 0x12345678)  # P == 0: output left untouched (mm:463-467)
    assert np.all(gpu["ranges"] == 0)
    # everything behind the camera
    g = scene.synthetic_gaussians(500, 3, w, h)
    g[:, 2] = -1.0
    ref = _oracle().forward(g, u, w, h)
    gpu = run_gpu(g, u, w, h, gt=np.zeros((h, w), np.uint32))
    compare_forward(gpu, ref)
    assert ref.num_pairs == 0
    assert np.all(gpu["grad"] == 0.0)


def test_edge_cases_mix(dev):
    """NaN / huge positions, degenerate quaternions, huge splats (tiny conic, > 256 tiles),
    saturated colours and opacities."""
    w, h = 256, 256
    g = scene.synthetic_gaussians(4000, 21, w, h)
    rng = np.random.default_rng(5)
    idx = rng.choice(4000, 400, replace=False)
    g[idx[:40], 0] = np.nan
    g[idx[40:80], 1] = 2e6
    g[idx[80:120], 8:12] = 0.0            # zero quaternion -> identity
    g[idx[120:160], 4:7] = 3.0            # huge splats (radius up to 512)
    g[idx[160:200], 4:7] = 8.0            # clamped at +5
    g[idx[200:240], 4] = -9.0             # extreme anisotropy (20:1 clamp)
    g[idx[240:280], 12] = 20.0            # opacity clamp +8
    g[idx[280:320], 12] = -9.0            # opacity below the 0.005 filter
    g[idx[320:360], 13] = 5.0             # colour saturates at 1
    g[idx[360:400], 13] = -5.0            # colour saturates at 0
    u = scene.make_uniforms(w, h)
    gt = scene.synthetic_ground_truth(21, 0, w, h)
    o = _oracle()
    ref = o.forward(g, u, w, h)
    gpu = run_gpu(g, u, w, h, gt=gt)
    compare_forward(gpu, ref)
    gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt)
    gr2, shadow = o.backward_shadow(g, ref, ref.rgba8, gt)
    assert np.array_equal(gr, gr2, equal_nan=True)
    assert np.array_equal(sh, shadow, equal_nan=True)
    # the huge splats overflow the reference's float dSigma chain (NaN); the fp64 shadow is finite
    assert (~np.isfinite(gr) & np.isfinite(shadow)).any()
    compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd)


def test_capacity_growth_path(dev):
    """Reserve far below P: the forward reads P back and grows instead of dropping pairs."""
    g, u, gt = _case(30000, 200, 150, 9)
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    r = TiledRasterizer(16, 0)  # tiny initial capacity
    gpu = run_gpu(g, u, 200, 150, gt=gt, rast=r)
    ref = _oracle().forward(g, u, 200, 150)
    compare_forward(gpu, ref)
    assert r.frame_stats()["pair_capacity"] >= ref.num_pairs


def test_deterministic(dev):
    g, u, gt = _case(8000, 256, 256, 13)
    a = run_gpu(g, u, 256, 256, gt=gt)
    b = run_gpu(g, u, 256, 256, gt=gt)
    assert np.array_equal(a["grad"].view(np.uint32), b["grad"].view(np.uint32))
    assert np.array_equal(a["rgba8"], b["rgba8"])


def test_density_accumulate_and_apply(dev):
    import torch

    from gaussiansplatting_amd.rasterizer import DensityController
    o = _oracle()
    w, h = 128, 128
    g, u, gt = _case(6000, w, h, 17)
    gpu = run_gpu(g, u, w, h, gt=gt)
    grads = gpu["grad"]
    n = g.shape[0]
    dc = DensityController(n, 0)
    dc.set_scene_extent(2.0)
    dc.reset_accumulator(n)
    dgrad = torch.from_numpy(grads).cuda()
    acc = np.zeros(n, np.float32)
    cnt = np.zeros(n, np.uint32)
    pos = np.zeros((n, 3), np.float32)
    for _ in range(3):
        dc.accumulate_gradients(dgrad)
        o.density_accumulate(grads, acc, cnt, pos)
    a2, c2, p2 = dc.read(n)
    assert np.array_equal(c2, cnt)
    assert np.array_equal(a2.view(np.uint32), acc.view(np.uint32))
    assert np.array_equal(p2.view(np.uint32), pos.view(np.uint32))
    # apply at iteration 3600 (prune by screen size + densify) with a low threshold scene
    dg = torch.from_numpy(g).cuda()
    for it in (600, 3600):
        dc.reset_accumulator(n)
        dc.accumulate_gradients(dgrad)
        acc = np.zeros(n, np.float32)
        cnt = np.zeros(n, np.uint32)
        pos = np.zeros((n, 3), np.float32)
        o.density_accumulate(grads, acc, cnt, pos)
        new, st = dc.apply(dg, it, focal_length=128.0, image_width=128.0, avg_depth=4.0, seed=99)
        ref, markers, rst = o.density_apply(g, acc, cnt, it, 2.0, 128.0, 128.0, 4.0, 99)
        assert st == rst
        assert rst["num_cloned"] + rst["num_split"] > 0
        assert np.array_equal(new.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_config1_against_golden_fixture(dev):
    """GPU outputs on the committed config-1 inputs hash-equal the committed oracle outputs."""
    import hashlib
    import os

    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_cfg1.npz"))

    def sha(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    gpu = run_gpu(d["gaussians"], d["uniforms"], 256, 256, gt=d["gt"])
    assert gpu["num_pairs"] == int(d["num_pairs"])
    assert sha(gpu["keys"]) == str(d["sha_keys"])
    assert sha(gpu["values"]) == str(d["sha_values"])
    assert sha(gpu["ranges"]) == str(d["sha_ranges"])
    assert sha(gpu["last_idx"]) == str(d["sha_last_idx"])
    assert sha(gpu["rgba8"]) == str(d["sha_rgba8"])
    assert sha(gpu["rgb"]) == str(d["sha_rgb"])
    live = [o for _, o in scene.GRAD_FIELDS]
    gsum = gpu["grad"][:, live].astype(np.float64).sum(0)
    assert np.all(np.abs(gsum - d["grad_sum"]) <= 1e-4 * d["grad_abs_sum"] + 1e-12)


def test_density_statistics_write_roundtrip(dev):
    """gs_density_write (the multi-GPU statistics reduce writes the summed accumulators back)."""
    import torch
    from gaussiansplatting_amd.rasterizer import DensityController
    n = 5000
    dc = DensityController(n, 0)
    dc.reset_accumulator(n)
    grads = torch.randn((n, 28), dtype=torch.float32, device=dev) * 1e-3
    dc.accumulate_gradients(grads, n)
    acc, cnt, pos = dc.statistics(n)
    dc.set_statistics(acc * 2, cnt * 3, pos + 1, n)
    a2, c2, p2 = dc.statistics(n)
    torch.cuda.synchronize()
    assert torch.equal(a2, acc * 2) and torch.equal(c2, cnt * 3) and torch.equal(p2, pos + 1)
    dc.close()


@pytest.mark.parametrize("n", [1, 2047, 2048, 2049, 4097, 70_001])
def test_sweep_partition_edges(dev, n):
    """Single-sweep depth sort and look-back offset scan at partition boundaries (2048 ranks per
    partition): one partial partition, exact multiples, one element over, many partitions."""
    w, h = 160, 120
    g, u, gt = _case(n, w, h, 31 + n % 7)
    gpu, ref = _full(g, u, gt, w, h)
    assert gpu["num_pairs"] == ref.num_pairs


def test_sweep_repeated_frames(dev):
    """The sweep's tickets and status words are re-armed every frame: frames 2 and 3 on the same
    handle (different N, then the first N again) equal fresh runs."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h = 320, 240
    r = TiledRasterizer(50_000, 0)
    for n, seed in [(50_000, 3), (7_000, 4), (50_000, 3)]:
        g, u, gt = _case(n, w, h, seed)
        o = _oracle()
        ref = o.forward(g, u, w, h)
        gpu = run_gpu(g, u, w, h, gt=gt, rast=r, backward=False)
        compare_forward(gpu, ref)


@pytest.mark.gpu
def test_float_exp_exhaustive():
    """The forward's float T_final track uses the hardware exp; its break window
    (gs_blend.hip tfinal_track_bound) assumes the hardware weight within kExpRelErr = 4e-7 of the
    pinned exp for every float power in [-4.5, 0]."""
    import ctypes

    from gaussiansplatting_amd import _lib

    L = _lib.lib()
    rel = ctypes.c_float(-1.0)
    _lib.check(L.gs_debug_float_exp_check(0, ctypes.byref(rel)), "float exp check")
    print(f"max relative difference hardware vs pinned exp over [-4.5, 0]: {rel.value:.3e}")
    assert 0.0 <= rel.value <= 4.0e-7


@pytest.mark.gpu
def test_half_exp_exhaustive():
    """The forward's half weight uses the hardware exp with no pinned fallback: over every half power in [-4.5, 0] the hardware exp must round to
    the same half as the pinned exp (gs_device.hpp gs_expf_core, the oracle's exp)."""
    import ctypes

    from gaussiansplatting_amd import _lib

    L = _lib.lib()
    mism, ulps = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _lib.check(L.gs_debug_half_exp_check(0, ctypes.byref(mism), ctypes.byref(ulps)), "half exp check")
    assert mism.value == 0, f"{mism.value} half powers round differently (max {ulps.value} ulps apart)"
    assert ulps.value <= 16



def test_stale_partial_slots_across_frames(dev):
    """Slots the backward does not reach are never written: their frame tag is stale and the chain
    ignores them (gs_internal.hpp kScalarFrameTag). Frames of different scenes on one handle reuse
    the same slots for different (tile, Gaussian) pairs; each frame's gradients must still equal
    the oracle's, including a frame with far fewer reached slots after a dense one, and a second
    backward of the same forward."""
    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h = 256, 192
    r = TiledRasterizer(40_000, 0)
    o = _oracle()
    for n, seed in [(40_000, 11), (6_000, 12), (40_000, 13)]:
        g, u, gt = _case(n, w, h, seed)
        ref = o.forward(g, u, w, h)
        gpu = run_gpu(g, u, w, h, gt=gt, rast=r)
        compare_forward(gpu, ref)
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gt)
        compare_gradients(gpu["grad"], gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=f"frame n={n} seed={seed}")
    # a second backward of the last forward with another ground truth: same reached slots
    import torch
    gt2 = scene.synthetic_ground_truth(99, 0, w, h)
    dev0 = torch.device("cuda:0")
    dg = torch.from_numpy(np.ascontiguousarray(g)).to(dev0)
    out = torch.empty((h, w), dtype=torch.int32, device=dev0)
    r.forward(dg, u, out)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev0)
    for gtx in (gt, gt2):
        r.backward(dg, grad, u, out, torch.from_numpy(gtx.view(np.int32)).to(dev0))
        torch.cuda.synchronize()
        gr, ab, nz, sh, cd = o.backward_full(g, ref, ref.rgba8, gtx)
        compare_gradients(grad.cpu().numpy(), gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="second backward of one forward")


def test_graph_replay_new_scene(dev):
    """A HIP graph of forward + backward replayed with new Gaussian contents in the same buffer:
    the frame tag is bumped on the device inside the graph, so the slots the new scene does not
    reach (but the captured one did) are not mixed into its gradients."""
    import torch

    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h, n = 256, 192, 30_000
    dev0 = torch.device("cuda:0")
    g1, u, gt = _case(n, w, h, 21)
    g2 = scene.synthetic_gaussians(n, 22, w, h)
    g2[::3, scene.G_OPACITY] = -9.0  # a third of the second scene nearly transparent (raw opacity): fewer reached slots
    r = TiledRasterizer(n, 0, w, h)
    r.reserve_pairs(n * min(256, scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]))  # sync-free
    dg = torch.from_numpy(np.ascontiguousarray(g1)).to(dev0)
    out = torch.empty((h, w), dtype=torch.int32, device=dev0)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev0)
    dgt = torch.from_numpy(gt.view(np.int32)).to(dev0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):  # warm up (allocations, reorder state) outside the capture
            r.forward(dg, u, out, stream=s)
            r.backward(dg, grad, u, out, dgt, stream=s)
        s.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            r.forward(dg, u, out, stream=s)
            r.backward(dg, grad, u, out, dgt, stream=s)
    o = _oracle()
    for gx in (g1, g2, g1):
        dg.copy_(torch.from_numpy(np.ascontiguousarray(gx)).to(dev0))
        graph.replay()
        torch.cuda.synchronize()
        ref = o.forward(gx, u, w, h)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.rgba8)
        gr, ab, nz, sh, cd = o.backward_full(gx, ref, ref.rgba8, gt)
        compare_gradients(grad.cpu().numpy(), gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="graph replay")


def test_reached_tag_wraps(dev):
    """The per-Gaussian reached tags keep the frame tag's low byte (gs_internal.hpp reach_t): 256
    frames after a dense scene, the Gaussians a sparser scene no longer reaches carry a matching
    byte again. The chain must then still find their slots stale by the slots' 32-bit tags: every
    replay of the sparse scene, over more than 256 frames, gives the same gradients, equal to the
    oracle's."""
    import torch

    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h, n = 128, 96, 4_000
    dev0 = torch.device("cuda:0")
    g1, u, gt = _case(n, w, h, 31)
    g2 = g1.copy()
    g2[::2, scene.G_OPACITY] = -9.0  # half of the scene nearly transparent: reached in g1, not in g2
    r = TiledRasterizer(n, 0, w, h)
    r.reserve_pairs(n * min(256, scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]))
    dg = torch.from_numpy(np.ascontiguousarray(g1)).to(dev0)
    d2 = torch.from_numpy(np.ascontiguousarray(g2)).to(dev0)
    out = torch.empty((h, w), dtype=torch.int32, device=dev0)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev0)
    dgt = torch.from_numpy(gt.view(np.int32)).to(dev0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):
            r.forward(dg, u, out, stream=s)
            r.backward(dg, grad, u, out, dgt, stream=s)
        s.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            r.forward(dg, u, out, stream=s)
            r.backward(dg, grad, u, out, dgt, stream=s)
    graph.replay()  # the dense frame: every Gaussian with a visible footprint reached
    torch.cuda.synchronize()
    dg.copy_(d2)
    graph.replay()
    torch.cuda.synchronize()
    first = grad.clone()
    o = _oracle()
    ref = o.forward(g2, u, w, h)
    gr, ab, nz, sh, cd = o.backward_full(g2, ref, ref.rgba8, gt)
    compare_gradients(first.cpu().numpy(), gr, ab, nz, shadow_ref=sh, cond_ref=cd, label="sparse frame")
    for k in range(300):
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(grad, first), f"sparse frame {k + 2} after the dense one differs"


def test_backward_step_fused_equals_unfused(dev):
    """gs_backward_step (chain -> density statistics -> Adam in one kernel) == gs_backward_packed +
    gs_density_accumulate_rows + gs_adam_step_rows, bit for bit: the Gaussians, both Adam moments and
    the density statistics after three training steps (moments non-zero from the second), with the
    plain and the compacting chain kernels, and without density statistics."""
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer, DensityController, TiledRasterizer
    w, h, n = 320, 180, 20_000
    g, u, gt = _case(n, w, h, 41)
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    lrs = (0.0016, 0.05, 0.01, 0.5, 0.025)  # 10x the defaults: the steps move the scene visibly
    for compact in (0, 1):
        for with_density in (True, False):
            runs = []
            for fused in (False, True):
                r = TiledRasterizer(n, 0)
                r.set_chain_compact(compact)
                adam = AdamOptimizer(n, 0)
                dens = DensityController(n, 0) if with_density else None
                if dens is not None:
                    dens.reset_accumulator(n)
                dg = torch.from_numpy(g.copy()).to(dev)
                out = torch.empty((h, w), dtype=torch.int32, device=dev)
                rows = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
                vs = torch.empty((n, 2), dtype=torch.float32, device=dev)
                for _ in range(3):
                    r.forward(dg, u, out)
                    if fused:
                        r.backward_step(dg, u, out, dgt, adam, dens, lrs)
                    else:
                        r.backward_rows(dg, rows, vs, u, out, dgt)
                        if dens is not None:
                            dens.accumulate_rows(rows, vs, n)
                        adam.step_rows(dg, rows, lrs, 0, n)
                torch.cuda.synchronize()
                m, v = adam.state(n)
                runs.append((dg.cpu().numpy(), m, v, dens.read(n) if dens is not None else None, adam.timestep))
                r.close()
            (ga, ma, va, da, ta), (gb, mb, vb, db, tb) = runs
            label = f"compact={compact} density={with_density}"
            assert ta == tb == 3, label
            assert not np.array_equal(ga, g), label  # the steps changed the scene
            assert np.array_equal(ga.view(np.uint32), gb.view(np.uint32)), f"{label}: Gaussians differ"
            assert np.array_equal(ma.view(np.uint32), mb.view(np.uint32)), f"{label}: first moments differ"
            assert np.array_equal(va.view(np.uint32), vb.view(np.uint32)), f"{label}: second moments differ"
            if with_density:
                for x, y in zip(da, db):
                    assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), label
                assert int(da[1].sum()) > 0, label


def test_backward_step_fused_cold_lanes_and_late_live(dev):
    """The fused step's shortcuts on states they skip work for: the cold SH moment lanes
    made non-zero before the fused steps -- by a records step whose gradients carry higher-SH fields,
    or by a written state -- and a block of Gaussians that no pixel reaches in the first step (raw
    opacity -9) and that becomes visible for the next two, so their live flags turn on inside the
    fused kernel. gs_backward_step must equal gs_backward_packed + gs_density_accumulate_rows +
    gs_adam_step_rows bit for bit (Gaussians, both moments, density statistics), with both chain
    kernels."""
    import torch

    from gaussiansplatting_amd.rasterizer import AdamOptimizer, DensityController, TiledRasterizer
    w, h, n = 320, 180, 20_000
    g, u, gt = _case(n, w, h, 43)
    late = slice(5_000, 9_000)
    g0 = g.copy()
    g0[late, scene.G_OPACITY] = -9.0
    dgt = torch.from_numpy(np.ascontiguousarray(gt).view(np.int32)).to(dev)
    lrs = (0.0016, 0.05, 0.01, 0.5, 0.025)
    rng = np.random.default_rng(7)
    grec = (rng.standard_normal((n, 28)) * 1e-2).astype(np.float32)  # every field, higher SH included
    mst = (np.abs(rng.standard_normal((n, 24))) * 1e-3).astype(np.float32)
    grec[late] = 0.0  # the hidden block keeps zero moments (live flag 0) until a pixel reaches it
    mst[late] = 0.0
    for compact in (0, 1):
        for cold in ("records", "state"):
            runs = []
            for fused in (False, True):
                r = TiledRasterizer(n, 0)
                r.set_chain_compact(compact)
                adam = AdamOptimizer(n, 0)
                dens = DensityController(n, 0)
                dens.reset_accumulator(n)
                dg = torch.from_numpy(g0.copy()).to(dev)
                if cold == "records":
                    adam.step(dg, torch.from_numpy(grec).to(dev), lrs)
                else:
                    ms = torch.from_numpy(mst).to(dev)
                    adam.set_state(ms, ms * ms, n)
                out = torch.empty((h, w), dtype=torch.int32, device=dev)
                rows = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
                vs = torch.empty((n, 2), dtype=torch.float32, device=dev)
                for k in range(3):
                    if k == 1:  # the hidden block becomes visible
                        dg[late, scene.G_OPACITY] = torch.from_numpy(g[late, scene.G_OPACITY]).to(dev)
                    r.forward(dg, u, out)
                    if fused:
                        r.backward_step(dg, u, out, dgt, adam, dens, lrs)
                    else:
                        r.backward_rows(dg, rows, vs, u, out, dgt)
                        dens.accumulate_rows(rows, vs, n)
                        adam.step_rows(dg, rows, lrs, 0, n)
                torch.cuda.synchronize()
                m, v = adam.state(n)
                runs.append((dg.cpu().numpy(), m, v, dens.read(n)))
                r.close()
                adam.close()
                dens.close()
            (ga, ma, va, da), (gb, mb, vb, db) = runs
            label = f"compact={compact} cold={cold}"
            assert (ma[:, 15:] != 0).any(), label  # the cold lanes are live
            assert (ma[late] != 0).any(axis=1).mean() > 0.5, label  # the late block stepped into life
            assert np.array_equal(ga.view(np.uint32), gb.view(np.uint32)), f"{label}: Gaussians differ"
            assert np.array_equal(ma.view(np.uint32), mb.view(np.uint32)), f"{label}: first moments differ"
            assert np.array_equal(va.view(np.uint32), vb.view(np.uint32)), f"{label}: second moments differ"
            for x, y in zip(da, db):
                assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), label


def test_graph_backwards_of_one_forward(dev):
    """The list split's hand-over words carry the frame tag and are cleared by the front quarter
    that consumes them (gs_blend.hip), so backwards of one forward in any mix of eager calls and
    HIP-graph replays never read each other's words: an eager forward, then a captured backward-only
    graph (another ground truth)
    replayed between eager backwards, and a graph of forward + two backwards. Every backward's
    gradients equal the oracle's for its own ground truth."""
    import torch

    from gaussiansplatting_amd.rasterizer import TiledRasterizer
    w, h, n = 256, 192, 30_000
    dev0 = torch.device("cuda:0")
    g, u, gt1 = _case(n, w, h, 51)
    gt2 = scene.synthetic_ground_truth(77, 0, w, h)
    r = TiledRasterizer(n, 0, w, h)
    r.reserve_pairs(n * min(256, scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]))
    dg = torch.from_numpy(np.ascontiguousarray(g)).to(dev0)
    out = torch.empty((h, w), dtype=torch.int32, device=dev0)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev0)
    grad2 = torch.empty((n, 28), dtype=torch.float32, device=dev0)
    d1 = torch.from_numpy(gt1.view(np.int32)).to(dev0)
    d2 = torch.from_numpy(gt2.view(np.int32)).to(dev0)
    o = _oracle()
    ref = o.forward(g, u, w, h)
    refs = {}
    for name, gtx in (("gt1", gt1), ("gt2", gt2)):
        refs[name] = o.backward_full(g, ref, ref.rgba8, gtx)

    def check(t, name, label):
        gr, ab, nz, sh, cd = refs[name]
        compare_gradients(t.cpu().numpy(), gr, ab, nz, shadow_ref=sh, cond_ref=cd, label=label)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        r.forward(dg, u, out, stream=s)
        r.backward(dg, grad, u, out, d1, stream=s)  # eager: allocates the split state
        s.synchronize()
        bwd_graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(bwd_graph, stream=s):
            r.backward(dg, grad2, u, out, d2, stream=s)
        r.forward(dg, u, out, stream=s)
        for k in range(2):
            bwd_graph.replay()
            s.synchronize()
            check(grad2, "gt2", f"graph backward {k}")
            r.backward(dg, grad, u, out, d1, stream=s)
            s.synchronize()
            check(grad, "gt1", f"eager backward {k} after a graph backward")
        both = torch.cuda.CUDAGraph()
        with torch.cuda.graph(both, stream=s):
            r.forward(dg, u, out, stream=s)
            r.backward(dg, grad, u, out, d1, stream=s)
            r.backward(dg, grad2, u, out, d2, stream=s)
        for k in range(2):
            both.replay()
            s.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.rgba8)
            check(grad, "gt1", f"graph forward + backward {k}")
            check(grad2, "gt2", f"graph second backward {k}")
    r.close()
