#!/usr/bin/env python3
"""bench_configs.py — the non-headline configurations of BASELINE.json (bench.py is config 3/4).

  --config 2   100k Gaussians initialised from a synthetic COLMAP scene (gaussiansFromColmap:
               large isotropic splats), view 0 at 1080p, forward only, 1 GPU.
  --config 5   5M Gaussians, full training step per GPU view: forward + loss (L1 + D-SSIM) +
               backward + density accumulate + Adam, and at N > 1 the RCCL all-reduce of the packed
               gradients. One density apply (iteration 600) runs during warm-up, so the timed steps
               see the densified population.

One JSON line per run, same fields as bench.py (value = Gaussians x views / s over all ranks).
  python bench_configs.py --config 5 [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench_configs.py --config 5 --gpus N
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, choices=(2, 5), required=True)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gaussians", type=int, default=0, help="override the config's N")
    ap.add_argument("--dist-backend", default="nccl")
    ap.add_argument("--records", action="store_true",
                    help="config 5: GaussianGradients records between backward, density and Adam (the "
                         "reference's data flow) instead of 56-B gradient rows")
    ap.add_argument("--unfused", action="store_true",
                    help="config 5, one GPU: gradient rows through gs_backward_packed, then density and Adam "
                         "as their own launches, instead of gs_backward_step (bit-identical)")
    ap.add_argument("--sharded-adam", action="store_true",
                    help="config 5, N > 1: reduce-scatter the rows, Adam on the rank's shard, all-gather "
                         "the Gaussians, instead of all-reduce + replicated Adam")
    ap.add_argument("--sync-capacity", action="store_true",
                    help="config 5: keep the pair reserve at 16 N (each frame reads P back to size the buffers) "
                         "instead of the worst case N min(256, T)")
    ap.add_argument("--depth-sort", type=int, default=0,
                    help="0 automatic, 1 global depth sort, 2 per-tile depth sort (gs_set_depth_sort)")
    ap.add_argument("--serial-loss", action="store_true",
                    help="config 5: the loss kernels on the launch stream between the forward and the backward, "
                         "instead of on a second stream beside the backward (the backward does not read the loss)")
    ap.add_argument("--tile-sort-path", type=int, default=0,
                    help="0 automatic, 1 one-pass counting sort, 2 two-pass LSD (gs_set_tile_sort_path)")
    args = ap.parse_args()

    from gaussiansplatting_amd import launch
    rc = launch.maybe_spawn(os.path.abspath(__file__), sys.argv[1:], args.gpus)
    if rc is not None:  # this process started the N ranks (bench.py does the same)
        return rc
    world = launch.check_world(args.gpus)

    import torch
    import torch.distributed as dist

    from gaussiansplatting_amd import _lib, io, multiview, scene
    from gaussiansplatting_amd.rasterizer import (AdamOptimizer, DensityController, Loss,
                                                  TiledRasterizer, _stream_ptr)

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device(f"cuda:{local_dev}")
    if world > 1:
        with launch.stdout_to_stderr():  # (RCCL's version banner: stdout is the JSON line's)
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(args.dist_backend)
            dist.barrier()
    cfg = scene.CONFIGS[args.config]
    n = args.gaussians or cfg["n"]
    w, h, seed = cfg["width"], cfg["height"], cfg["seed"]
    view = rank % 8
    L = _lib.lib()

    if args.config == 2:
        with tempfile.TemporaryDirectory() as d:
            io.synthetic_colmap(d, n, seed, w, h, views=8)
            sc = io.load_colmap(d)
            g = sc.gaussians()
            u = sc.uniforms(view, w, h)
            extent = sc.scene_extent()
            sc.close()
    else:
        g = scene.synthetic_gaussians(n, seed, w, h)
        u = scene.rig_uniforms(view, w, h)
        extent = 1.1 * 0.25 * 3.5  # the rig's camera spread (cameras at 0.25 (j - 3.5))
    gt = scene.synthetic_ground_truth(seed, view, w, h)
    tiles = scene.tiles_for(w, h)[0] * scene.tiles_for(w, h)[1]
    ubuf = (ctypes.c_float * 60).from_buffer_copy(np.ascontiguousarray(u).tobytes())

    cap_n = 2 * n  # densification can grow the population
    dg = torch.zeros((cap_n, 28), dtype=torch.float32, device=dev)
    dg[:n] = torch.from_numpy(g).to(dev)
    dgt = torch.from_numpy(gt.view(np.int32)).to(dev)
    out = torch.empty((h, w), dtype=torch.int32, device=dev)
    grad = torch.empty((cap_n, 28), dtype=torch.float32, device=dev)
    rows = torch.empty((cap_n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    vs = torch.empty((cap_n, 2), dtype=torch.float32, device=dev)
    loss_out = torch.empty(1, dtype=torch.float32, device=dev)
    rast = TiledRasterizer(cap_n, local_dev, w, h)
    rast.reserve_pairs(n * 16 if args.config == 5 else n * min(256, tiles))
    hh = rast._h
    rast.set_tile_sort_path(args.tile_sort_path)
    rast.set_depth_sort(args.depth_sort)
    state = {"n": n}
    lrs = (0.00016, 0.005, 0.001, 0.025, 0.0025)  # mtl_engine.mm:1060-1069
    lrs_c = (ctypes.c_float * 5)(*lrs)

    if args.config == 5:
        loss = Loss(local_dev)
        adam = AdamOptimizer(cap_n, local_dev)
        dc = DensityController(0, local_dev)
        dc.set_scene_extent(extent)
        dc.reset_accumulator(n)

    def fwd(st):
        _lib.check(L.gs_forward(hh, st, dg.data_ptr(), state["n"], ubuf, w, h, out.data_ptr(), None), "gs_forward")

    # The loss (L1 + D-SSIM of the render against the ground truth, mtl_engine.mm:769-853) only feeds
    # the reported loss value: the reference's backward takes dL/dpixel = sign(r - gt) / 3 itself
    # (tiled_shaders.metal:418-423). So it runs on a second stream beside the backward, ordered after
    # the forward (it reads the render) and joined before the step ends (the next forward overwrites
    # the render): the same kernels, overlapped with the backward instead of between it and the forward.
    side = torch.cuda.Stream(device=dev) if args.config == 5 and not args.serial_loss else None

    def train_step():
        st = _stream_ptr(None)
        nn = state["n"]
        fwd(st)
        joined = None
        if side is not None:
            rendered = torch.cuda.Event()
            rendered.record()
            side.wait_event(rendered)
            loss.compute(out, dgt, 0.2, out=loss_out, stream=side)
            joined = torch.cuda.Event()
            joined.record(side)
        else:
            loss.compute(out, dgt, 0.2, out=loss_out)
        try:
            train_rest(st, nn)
        finally:
            if joined is not None:
                torch.cuda.current_stream().wait_event(joined)

    def train_rest(st, nn):
        if args.records:  # the reference's data flow: GaussianGradients records (112 B per Gaussian)
            _lib.check(L.gs_backward(hh, st, dg.data_ptr(), grad.data_ptr(), nn, ubuf, out.data_ptr(),
                                     dgt.data_ptr()), "gs_backward")
            dc.accumulate_gradients(grad, nn)
            if world > 1:
                raise SystemExit("--records is the single-GPU reference data flow")
            _lib.check(L.gs_adam_step(adam._h, _stream_ptr(None), dg.data_ptr(), grad.data_ptr(), nn, lrs_c),
                       "gs_adam_step")
            return
        if world == 1 and not args.unfused:
            # chain -> density statistics -> Adam per Gaussian in one kernel: no gradient rows at all
            rast.backward_step(dg[:nn], u, out, dgt, adam, dc, lrs)
            return
        # gradient rows (56 B) + per-view viewspace rows (8 B): the records are never written
        _lib.check(L.gs_backward_packed(hh, st, dg.data_ptr(), rows.data_ptr(), vs.data_ptr(), nn, ubuf,
                                        out.data_ptr(), dgt.data_ptr()), "gs_backward_packed")
        # density statistics from this rank's own view, before any reduce
        dc.accumulate_rows(rows, vs, nn)
        if world == 1:
            adam.step_rows(dg, rows, lrs, 0, nn)
        elif args.sharded_adam:
            # reduce-scatter -> Adam on this rank's shard -> all-gather of the updated Gaussians
            multiview.sharded_adam_step(adam, dg, rows, nn, lrs)
        else:
            multiview.reduce_gradients(rows[:nn])
            adam.step_rows(dg, rows, lrs, 0, nn)

    step = (lambda: fwd(_stream_ptr(None))) if args.config == 2 else train_step
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    applied = None
    if args.config == 5:  # one densification (iteration 600) before the timed steps
        n0 = state["n"]
        # replicas densify identically: the per-rank statistics are summed first
        multiview.reduce_density_statistics(lambda: dc.statistics(n0),
                                             lambda a, c, p: dc.set_statistics(a, c, p, n0))
        if world > 1 and args.sharded_adam:  # each rank stepped its own shard's moments
            multiview.gather_adam_state(adam, n0)
        new, stats = dc.apply(dg[:n0], 600, focal_length=float(w), image_width=float(w), avg_depth=6.0,
                              seed=600)
        n1 = min(int(new.shape[0]), cap_n)
        dg[:n1] = new[:n1]
        adam.follow_density(dc, n0, int(new.shape[0]))
        state["n"] = n1
        dc.reset_accumulator(n1)
        # the pair buffers at the worst case for the timed population (N min(256, T): 1.33G pairs,
        # 86 GB of the 288 GB HBM3E), as bench.py reserves for its 1M Gaussians: no frame then reads P
        # back to size them (gs_reserve_pairs; a 4-B readback and a host round trip per frame below it)
        if not args.sync_capacity:
            rast.reserve_pairs(n1 * min(256, tiles))
        applied = dict(stats, n_before=n0, n_after=n1)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-stage breakdown of the rasterizer (hipEvents on the launch stream), from separate steps
    ms_buf = (ctypes.c_double * 16)()
    calls_buf = (ctypes.c_uint32 * 16)()
    L.gs_set_stage_timing(hh, 1)
    L.gs_stage_times(hh, ms_buf, calls_buf, 16)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    nst = L.gs_stage_times(hh, ms_buf, calls_buf, 16)
    stage_ms = {name: ms_buf[i] / max(1, calls_buf[i]) for i, name in enumerate(_lib.STAGES[:nst])}
    L.gs_set_stage_timing(hh, 0)
    stats = rast.frame_stats()
    tr = torch.empty((tiles, 2), dtype=torch.int32, device=dev)  # the last frame's tile lists
    _lib.check(L.gs_debug_tile_ranges(hh, _stream_ptr(None), tr.data_ptr(), tiles), "gs_debug_tile_ranges")
    lens = tr.cpu().numpy().view(np.uint32)[:, 1].astype(np.int64)
    nn = state["n"]
    res = {
        "metric": ("Gaussians*views/s fwd @1080p (cfg2, COLMAP-initialised)" if args.config == 2 else
                   "Gaussians*views/s full train step @1080p (cfg5)"),
        "value": nn * world / (elapsed / args.steps),
        "unit": "Gaussians*views/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic" + (" COLMAP scene (io.synthetic_colmap)" if args.config == 2 else " (SURVEY.md §8d)"),
        "config": {"workload": f"cfg{args.config}: {nn} Gaussians, {w}x{h}, view {view} per GPU",
                   "gaussians": nn, "pairs_per_view": int(stats["num_pairs"]),
                   "pair_capacity": int(stats["pair_capacity"]),
                   "step": "forward" if args.config == 2 else
                           "forward + loss + backward + density accumulate + Adam" +
                           (" (GaussianGradients records)" if args.records else
                            " (fused per Gaussian: gs_backward_step)" if world == 1 and not args.unfused else
                            " (56-B gradient rows)") +
                           ((" + RCCL reduce-scatter, sharded Adam, all-gather" if args.sharded_adam else
                             " + RCCL all-reduce") if world > 1 else ""),
                   "density_apply": applied,
                   "tile_lists": {"max": int(lens.max()), "p50": int(np.quantile(lens, 0.5)),
                                  "p99": int(np.quantile(lens, 0.99)),
                                  "over_1024": int((lens > 1024).sum()), "over_4096": int((lens > 4096).sum())}},
        "stage_ms": stage_ms,
        # the last frame's work counters (GsFrameStats): the list entries the blends walked, the
        # Gaussians the backward reached and their slots (scripts/pmc_traffic.py --facts)
        "work": {k: int(stats[k]) for k in ("fwd_walked_entries", "bwd_walked_entries", "reached_gaussians",
                                            "reached_slots")},
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    rast.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
