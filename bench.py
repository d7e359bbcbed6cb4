#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Gaussians x views / s, forward + backward @ 1080p on MI355X,
with achieved HBM GB/s against the roofline.

One step = one view per GPU: TiledRasterizer forward (project -> keys -> sort -> ranges -> blend)
+ backward (blend backward -> per-Gaussian chain) and, at N > 1 GPUs, the RCCL all-reduce of the
packed per-Gaussian gradients (64 B per Gaussian) + unpack into GaussianGradients records.
Workload (configs[2] / configs[3] of BASELINE.json): 1M synthetic Gaussians (SURVEY.md §8d,
seed 3), 1920x1080, rank r renders camera r of the 8-camera rig. Inputs are resident in HBM
before the timed region. Weak scaling: every GPU renders one view per step.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(n: int, p: int, npix: int, tiles: int, k: int) -> dict:
    """Compulsory HBM bytes per view."""
    return {
        "project": 56 * n + 76 * n,
        "pairs": 24 * n + 12 * p,
        "sort": 24 * k * p,
        "ranges": 8 * p + 8 * tiles,
        "forward_blend": 40 * p + 8 * tiles + 8 * npix,
        "backward_blend": 40 * p + 8 * tiles + 12 * npix,
        "chain": 68 * n + 64 * n,
        "total": 288 * n + (100 + 24 * k) * p + 20 * npix + 24 * tiles,
    }


STAGE_BYTES_KEY = {
    "project": "project", "depth_sort": None, "offset_scan": None, "pair_emit": "pairs",
    "tile_sort": "sort", "tile_ranges": "ranges", "forward_blend": "forward_blend",
    "backward_blend": "backward_blend", "chain": "chain",
}


def cpu_baseline(n, w, h, seed, threads):
    """The oracle (CPU restatement of the reference kernels) on one full view of the same
    workload: forward + backward, `threads` OpenMP threads."""
    from gaussiansplatting_amd import scene
    from oracle import oracle
    g = scene.synthetic_gaussians(n, seed, w, h)
    u = scene.rig_uniforms(0, w, h)
    gt = scene.synthetic_ground_truth(seed, 0, w, h)
    t0 = time.perf_counter()
    f = oracle.forward(g, u, w, h, threads=threads)
    oracle.backward(g, f, f.rgba8, gt, threads=threads, stats=False)
    dt = time.perf_counter() - t0
    # the reference's own CPU stage (parallelRadixSort, tiled_rasterizer.mm:27-102) at its native
    # NUM_THREADS = 8 on this view's pairs
    keys, vals = f.keys.copy(), f.values.copy()
    rng = np.random.default_rng(0)
    perm = rng.permutation(keys.size)
    keys, vals = keys[perm], vals[perm]
    t1 = time.perf_counter()
    oracle.sort_pairs(keys, vals, threads=8)
    ts = time.perf_counter() - t1
    return {"value": n / dt, "unit": "Gaussians*views/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"1 view of the benchmark workload ({n} Gaussians, {w}x{h}, rig view 0), "
                      f"oracle forward+backward, {dt:.2f} s",
            "reference_sort_8_threads_s": ts, "reference_sort_pairs": int(keys.size)}


def load_profile_value(fname: str, kernel: str, workload: str):
    try:
        with open(os.path.join(ROOT, "profiles", fname)) as fh:
            e = json.load(fh).get(workload, {}).get(kernel)
        return float(e) if e is not None else None
    except Exception:
        return None


def device_copy_gbs(torch, dev, nbytes: int = 1 << 31, reps: int = 5) -> float:
    """Measured device-to-device copy bandwidth (read + write bytes / s), SURVEY.md §8d."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbs


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def load_traffic(kernel: str, workload: str):
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        e = d.get(workload, {}).get(kernel)
        return float(e) if e is not None else None
    except Exception:
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch every kernel eagerly")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--reduce-chunks", type=int, default=4,
                    help="N > 1: chunks of the per-Gaussian chain whose all-reduce overlaps the next chunk")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm) on a multi-GPU node; gloo only to rehearse N>1 on one GPU")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from gaussiansplatting_amd import _lib, multiview, scene
    from gaussiansplatting_amd.rasterizer import TiledRasterizer, _stream_ptr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device(f"cuda:{local_dev}")
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    n, w, h, seed = args.gaussians, args.width, args.height, args.seed
    tx, ty = scene.tiles_for(w, h)
    tiles = tx * ty
    view = rank % 8
    g = scene.synthetic_gaussians(n, seed, w, h)
    u = scene.rig_uniforms(view, w, h)
    gt = scene.synthetic_ground_truth(seed, view, w, h)
    dg = torch.from_numpy(g).to(dev)
    dgt = torch.from_numpy(gt.view(np.int32)).to(dev)
    out = torch.empty((h, w), dtype=torch.int32, device=dev)
    packed = torch.empty((n, 16), dtype=torch.float32, device=dev)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev)
    ubuf = (ctypes.c_float * 60).from_buffer_copy(np.ascontiguousarray(u).tobytes())

    rast = TiledRasterizer(n, local_dev, w, h)
    rast.reserve_pairs(n * min(256, tiles))  # worst case: the frame never syncs to the host
    L = _lib.lib()
    hh = rast._h

    def compute():
        """The GPU work of one step on the current stream (everything but the collective)."""
        st = _stream_ptr(None)
        _lib.check(L.gs_forward(hh, st, dg.data_ptr(), n, ubuf, w, h, out.data_ptr(), None),
                   "gs_forward")
        if world == 1:  # GaussianGradients records straight from the chain kernel
            _lib.check(L.gs_backward(hh, st, dg.data_ptr(), grad.data_ptr(), n, ubuf,
                                     out.data_ptr(), dgt.data_ptr()), "gs_backward")
        else:  # blend only: the chain runs chunk by chunk under the all-reduce (finish)
            _lib.check(L.gs_backward_blend(hh, st, dg.data_ptr(), n, ubuf, out.data_ptr(),
                                           dgt.data_ptr()), "gs_backward_blend")

    def finish():
        if world > 1:
            # per chunk of Gaussians: the chain into 64-B packed rows, then its RCCL all-reduce over
            # xGMI (async, on the collective's stream) while the next chunk's chain runs; each
            # chunk's GaussianGradients records are unpacked once its reduce has landed
            st = _stream_ptr(None)

            def chain(a, b):
                _lib.check(L.gs_backward_chain(hh, st, dg.data_ptr(), None, packed.data_ptr(), n, ubuf,
                                               a, b - a), "gs_backward_chain")

            def unpack(a, b):
                _lib.check(L.gs_unpack_gradients(st, packed.data_ptr() + a * 64, grad.data_ptr() + a * 112,
                                                 b - a), "gs_unpack_gradients")

            multiview.pipelined_reduce(packed, args.reduce_chunks, chain, unpack)

    def eager_step():
        compute()
        finish()

    for _ in range(args.warmup):
        eager_step()
    torch.cuda.synchronize()
    step = eager_step
    graph = None
    if not args.no_graph:
        # the ~40 launches of a step replayed as one HIP graph: the frame is sync-free (pairs
        # reserved at the worst case), so the whole forward + backward is capturable
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            compute()
        torch.cuda.synchronize()

        def graph_step():
            graph.replay()
            finish()

        step = graph_step
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

    # per-stage breakdown (hipEvents on the launch stream) from separate eager steps, so the
    # event records do not perturb the timed region
    ms_buf = (ctypes.c_double * 16)()
    calls_buf = (ctypes.c_uint32 * 16)()
    L.gs_set_stage_timing(hh, 1)
    L.gs_stage_times(hh, ms_buf, calls_buf, 16)  # drop anything recorded so far
    for _ in range(args.steps):
        eager_step()
    torch.cuda.synchronize()
    nst = L.gs_stage_times(hh, ms_buf, calls_buf, 16)
    stage_ms = {name: ms_buf[i] / max(1, calls_buf[i]) for i, name in enumerate(_lib.STAGES[:nst])}
    stats = rast.frame_stats()
    p = int(stats["num_pairs"])
    L.gs_set_stage_timing(hh, 0)

    ms_per_step = 1e3 * elapsed / args.steps
    value = n * world / (elapsed / args.steps)
    k = (32 + max(1, (tiles - 1).bit_length()) + 7) // 8
    alg = algorithmic_bytes(n, p, w * h, tiles, k)
    # dominant single-kernel stage
    kernel_stages = ["project", "pair_emit", "tile_ranges", "forward_blend", "backward_blend", "chain"]
    dom = max(kernel_stages, key=lambda s: stage_ms.get(s, 0.0))
    dom_ms = stage_ms[dom]
    dom_bytes = alg[STAGE_BYTES_KEY[dom]]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    workload = f"{n}g_{w}x{h}"
    traffic = load_traffic(dom, workload)
    valu = load_profile_value("valu.json", dom, workload)
    valu_peak = 256 * 4 * 2.4e9 / 2.0  # wave64 VALU instr/s: 1024 SIMD-32s, 2 cycles each, 2.4 GHz
    pipeline_ms = sum(stage_ms.values())
    result = {
        "metric": "Gaussians*views/s fwd+bwd @1080p",
        "value": value,
        "unit": "Gaussians*views/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "precision_note": "forward blend in f16 (reference semantics, bit-exact), gradient chain in f64",
        "data": "synthetic (SURVEY.md §8d seeded scene, random RGBA8 ground truth)",
        "config": {"workload": f"cfg3/cfg4: {n} Gaussians, {w}x{h}, 1 view per GPU (rig camera = rank), "
                               "forward+backward" + (f" + RCCL all-reduce of packed gradients ({args.reduce_chunks} chunks overlapping the chain)" if world > 1 else ""),
                   "gaussians": n, "width": w, "height": h, "views_per_step": world,
                   "pairs_per_view": p, "parallelism": f"views sharded dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "alg_bytes_per_launch": dom_bytes,
                     "avg_launch_ms": dom_ms},
        "roofline_valu": {"bound": "valu", "kernel": dom,
                          "achieved": valu / (dom_ms * 1e-3) if (valu and dom_ms) else None,
                          "peak": valu_peak, "unit": "wave64 VALU instr/s",
                          "frac": valu / (dom_ms * 1e-3) / valu_peak if (valu and dom_ms) else None,
                          "valu_instr_per_launch": valu,
                          "note": "SQ_INSTS_VALU per launch from profiles/valu.json (rocprofv3 PMC); "
                                  "peak = 157.3 TFLOP/s FP32 vector / (64 lanes x 2 flops)"},
        "roofline_pipeline": {"alg_bytes_per_view": alg["total"],
                              "achieved_gbs": alg["total"] / (pipeline_ms * 1e-3) / 1e9 if pipeline_ms else 0.0,
                              "frac": (alg["total"] / (pipeline_ms * 1e-3) / 1e9) / HBM_PEAK_GBS if pipeline_ms else 0.0,
                              "kernel_ms_per_view": pipeline_ms},
        "stage_ms": stage_ms,
        "launch": "eager" if graph is None else "hip_graph",
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["hbm_copy_gbs"] = device_copy_gbs(torch, dev)
        result["cpu_baseline"] = cpu_baseline(n, w, h, seed, args.cpu_threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    rast.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
