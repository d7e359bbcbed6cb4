#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Gaussians x views / s, forward + backward @ 1080p on MI355X,
with achieved HBM GB/s against the roofline.

One step = one view per GPU: TiledRasterizer forward (project -> keys -> sort -> ranges -> blend)
+ backward (blend backward -> per-Gaussian chain) and, at N > 1 GPUs, the RCCL all-reduce of the
per-Gaussian gradient rows (56 B per Gaussian; the screen-space gradient stays per rank) + unpack
into GaussianGradients records.
Workload (configs[2] / configs[3] of BASELINE.json): 1M synthetic Gaussians (SURVEY.md §8d,
seed 3), 1920x1080, rank r renders camera r of the 8-camera rig. Inputs are resident in HBM
before the timed region. Weak scaling: every GPU renders one view per step.

  python bench.py [--gpus N] [--steps K] [--warmup W]   (N > 1: starts its own N ranks)
  torchrun --nproc-per-node N bench.py --gpus N ...      (WORLD_SIZE must equal --gpus)
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


def host_cpus() -> dict:
    """The host cores this process may use: the affinity mask, capped by a cgroup CPU quota (the
    GPU box shows every CPU of the machine in nproc but grants a share)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota,
            "threads": min(aff, quota) if quota else aff}


def build_native_oracle(dest_dir: str) -> str | None:
    """oracle/gs_oracle.c built -O3 -march=native for this host (BASELINE.md CPU-baseline plan) into
    `dest_dir` (a temporary directory the caller removes); None if no compiler is available (the
    prebuilt x86-64-v3 library is used)."""
    import subprocess
    out = os.path.join(dest_dir, "gs_oracle_native.so")
    cmd = ["gcc", "-O3", "-march=native", "-std=c11", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off",
           "-fno-fast-math", "-o", out, os.path.join(ROOT, "oracle", "gs_oracle.c"), "-lm"]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=180)
        return out
    except Exception:
        return None


def cpu_baseline(threads: int, reps: int = 3) -> dict:
    """BASELINE.md's CPU baseline: the oracle (the CPU restatement of the reference kernels; the
    reference has no CPU rasterizer) built -march=native, OpenMP over the host cores this process
    may use, on configs 1-3 (1: 10k Gaussians 256x256 fwd+bwd; 2: 100k COLMAP-initialised
    Gaussians 1080p fwd; 3: the benchmark workload, 1M Gaussians 1080p fwd+bwd), median of `reps`;
    plus the reference's own CPU stage (parallelRadixSort, tiled_rasterizer.mm:27-102) at its
    native NUM_THREADS = 8 on config 3's pairs."""
    import statistics
    import tempfile

    from gaussiansplatting_amd import io, scene
    from oracle import oracle
    default_lib = oracle.LIB_PATH
    with tempfile.TemporaryDirectory() as tmp:
        native = build_native_oracle(tmp)
        if native:
            oracle.use_library(native)
        try:
            return _cpu_baseline_runs(oracle, io, scene, statistics, tempfile, threads, reps, native)
        finally:
            oracle.use_library(default_lib)  # the module's default library for the rest of the process


def _cpu_baseline_runs(oracle, io, scene, statistics, tempfile, threads: int, reps: int, native) -> dict:
    per_cfg = {}
    f3 = None
    for cfg in (1, 2, 3):
        c = scene.CONFIGS[cfg]
        n, w, h, seed = c["n"], c["width"], c["height"], c["seed"]
        if cfg == 2:
            with tempfile.TemporaryDirectory() as d:
                io.synthetic_colmap(d, n, seed, w, h, views=8)
                sc = io.load_colmap(d)
                g, u = sc.gaussians(), sc.uniforms(0, w, h)
                sc.close()
        else:
            g = scene.synthetic_gaussians(n, seed, w, h)
            u = scene.rig_uniforms(0, w, h) if cfg == 3 else scene.make_uniforms(w, h)
        gt = scene.synthetic_ground_truth(seed, 0, w, h)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            f = oracle.forward(g, u, w, h, threads=threads)
            if cfg != 2:  # config 2 is forward only (BASELINE.json configs[1])
                oracle.backward(g, f, f.rgba8, gt, threads=threads, stats=False)
            times.append(time.perf_counter() - t0)
        med = statistics.median(times)
        per_cfg[f"cfg{cfg}"] = {"gaussians": n, "width": w, "height": h, "pairs": int(f.num_pairs),
                                "step": "forward" if cfg == 2 else "forward+backward",
                                "median_s": med, "runs_s": times, "gaussians_views_per_s": n / med}
        if cfg == 3:
            f3 = f
    keys, vals = f3.keys.copy(), f3.values.copy()
    perm = np.random.default_rng(0).permutation(keys.size)
    keys, vals = keys[perm], vals[perm]
    t1 = time.perf_counter()
    oracle.sort_pairs(keys, vals, threads=8)
    ts = time.perf_counter() - t1
    c3 = per_cfg["cfg3"]
    return {"value": c3["gaussians_views_per_s"], "unit": "Gaussians*views/s", "cores": threads,
            "kind": "port", "cpu_model": cpu_model(), "host": host_cpus(),
            "build": "gcc -O3 -march=native -fopenmp -ffp-contract=off" if native else
                     "prebuilt oracle/libgs_oracle.so (-O3 -march=x86-64-v3)",
            "sample": f"config 3 (the benchmark workload: {c3['gaussians']} Gaussians, {c3['width']}x{c3['height']}, "
                      f"rig view 0), oracle forward+backward, median of {reps}: {c3['median_s']:.2f} s",
            "configs": per_cfg,
            "reference_sort_8_threads_s": ts, "reference_sort_pairs": int(keys.size)}


def load_profile_value(fname: str, kernel: str, workload: str):
    try:
        with open(os.path.join(ROOT, "profiles", fname)) as fh:
            e = json.load(fh).get(workload, {}).get(kernel)
        return float(e) if e is not None else None
    except Exception:
        return None


def device_copy_gbs(L, device: int, nbytes: int = 1 << 31, reps: int = 10) -> dict:
    """Measured HBM copy bandwidth (read + write bytes / s), SURVEY.md §8d: the library's 16-B-per-lane
    streaming copy kernel (gs_membw.hip) over two 2-GiB buffers (past the 256 MiB Infinity Cache),
    plain and non-temporal at 1/2/4/8 workgroups per CU; the best of them."""
    from gaussiansplatting_amd import _lib
    best = ctypes.c_double(0.0)
    var = (ctypes.c_double * 8)()
    _lib.check(L.gs_debug_copy_bandwidth(device, nbytes, reps, ctypes.byref(best), var, 8), "gs_debug_copy_bandwidth")
    names = [f"{k}_{c}wg_per_cu" for k in ("plain", "nontemporal") for c in (1, 2, 4, 8)]
    return {"best_gbs": best.value, "bytes_per_buffer": nbytes, "kernel": "gs_membw.hip copy_stream_kernel",
            "variants_gbs": {n: v for n, v in zip(names, var)}}


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


def comm_fields(world: int, nbytes: int, exposed_ms: float, allreduce_ms: float, chunks: int,
                backend: str) -> dict:
    """The N > 1 communication record of the bench line: the step's exposed all-reduce time (the
    part of the per-chunk waits the chain did not hide, multiview.CommTimer) and a standalone
    all-reduce of the same packed buffer: algorithm bandwidth bytes / t and ring bus bandwidth
    2 (n - 1) / n * bytes / t (what each xGMI link carries)."""
    t = allreduce_ms * 1e-3
    algo = nbytes / t / 1e9 if t > 0 else 0.0
    bus = 2.0 * (world - 1) / world * algo if world > 1 else 0.0
    return {"backend": backend, "bytes_per_step": int(nbytes), "chunks": int(chunks),
            "allreduce_exposed_ms": exposed_ms, "allreduce_standalone_ms": allreduce_ms,
            "algo_gbs": algo, "bus_gbs": bus}


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
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every core this process may use)")
    ap.add_argument("--reduce-chunks", type=int, default=4,
                    help="N > 1: chunks of the per-Gaussian chain whose all-reduce overlaps the next chunk")
    ap.add_argument("--backward-split", type=int, default=-1,
                    help="tiles whose backward runs as two list halves (-1 automatic, 0 off)")
    ap.add_argument("--chain-compact", type=int, default=-1,
                    help="gs_set_chain_compact: -1 automatic, 0 plain chain, 1 screen + list chain")
    ap.add_argument("--depth-sort", type=int, default=0,
                    help="0 automatic, 1 global depth sort, 2 per-tile depth sort (gs_set_depth_sort)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm) on a multi-GPU node; gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--rccl-single-rank", action="store_true",
                    help="N = 1 only: run the N > 1 step shape (chunked chain + async RCCL all-reduce + "
                         "unpack) on a one-rank RCCL group, to exercise RCCL on a one-GPU box")
    args = ap.parse_args()
    if args.rccl_single_rank and args.gpus != 1:
        ap.error("--rccl-single-rank is a one-GPU rehearsal (--gpus 1)")

    from gaussiansplatting_amd import launch
    # `python bench.py --gpus N`: start the N ranks (one process per GPU) before anything here
    # touches the GPU, relay their output and exit with the worst rank's status
    rc = launch.maybe_spawn(os.path.abspath(__file__), sys.argv[1:], args.gpus)
    if rc is not None:
        return rc
    world = launch.check_world(args.gpus)  # a launcher's WORLD_SIZE must equal --gpus

    import torch
    import torch.distributed as dist

    from gaussiansplatting_amd import _lib, multiview, scene
    from gaussiansplatting_amd.rasterizer import TiledRasterizer

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_dev)
    dev = torch.device(f"cuda:{local_dev}")
    # RCCL prints its version banner on stdout when a communicator comes up: keep stdout for the one
    # JSON line (the banner goes to stderr)
    with launch.stdout_to_stderr():
        if world > 1:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(args.dist_backend)
            dist.barrier()
        elif args.rccl_single_rank:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(launch.free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
            dist.barrier()
    split = world > 1 or args.rccl_single_rank  # the step shape with the collective

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
    packed = torch.empty((n, scene.ROW_FLOATS), dtype=torch.float32, device=dev)
    grad = torch.empty((n, 28), dtype=torch.float32, device=dev)

    rast = TiledRasterizer(n, local_dev, w, h)
    rast.reserve_pairs(n * min(256, tiles))  # worst case: the frame never syncs to the host
    rast.set_backward_split(args.backward_split)
    rast.set_depth_sort(args.depth_sort)
    rast.set_chain_compact(args.chain_compact)
    L = _lib.lib()
    hh = rast._h
    # the rank's step (multiview.ViewStep): at N > 1 the chain runs chunk by chunk under the RCCL
    # all-reduce of the gradient rows (finish), everything before it is compute()
    vs = multiview.ViewStep(rast, dg, u, out, dgt, grad, packed if split else None, world=world,
                            chunks=args.reduce_chunks, split=split)
    compute, finish = vs.compute, vs.finish

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
    if split:
        vs.timer = multiview.CommTimer(cuda=True)
    for _ in range(args.steps):
        eager_step()
    torch.cuda.synchronize()
    nst = L.gs_stage_times(hh, ms_buf, calls_buf, 16)
    # per step (at N > 1 the chain runs as `reduce_chunks` calls per step)
    stage_ms = {name: ms_buf[i] / args.steps for i, name in enumerate(_lib.STAGES[:nst]) if calls_buf[i]}
    comm = None
    if split:
        exposed = vs.timer.mean_exposed_ms()
        nbytes = vs.timer.bytes_per_step
        vs.timer = None
        dist.barrier()
        torch.cuda.synchronize()
        ar0, ar1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        dist.all_reduce(packed)  # warm
        torch.cuda.synchronize()
        ar0.record()
        for _ in range(reps):
            dist.all_reduce(packed)
        ar1.record()
        torch.cuda.synchronize()
        comm = comm_fields(world, nbytes, exposed, ar0.elapsed_time(ar1) / reps, args.reduce_chunks,
                           args.dist_backend)
        stage_ms["allreduce_exposed"] = exposed
    stats = rast.frame_stats()
    p = int(stats["num_pairs"])
    walked = {k: int(stats[k]) for k in ("fwd_walked_entries", "bwd_walked_entries", "reached_gaussians",
                                         "reached_slots")}
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
    # the same formula over the list entries the blends actually walked (each stops at its pixels'
    # last contributor / saturation): the compulsory count, not the §8d upper bound over all P pairs
    walk_p = {"forward_blend": walked["fwd_walked_entries"], "backward_blend": walked["bwd_walked_entries"]}.get(dom)
    dom_walked = algorithmic_bytes(n, walk_p, w * h, tiles, k)[STAGE_BYTES_KEY[dom]] if walk_p is not None else None
    achieved_walked = dom_walked / (dom_ms * 1e-3) / 1e9 if (dom_walked and dom_ms > 0) else None
    workload = f"{n}g_{w}x{h}"
    traffic = load_traffic(dom, workload)
    valu = load_profile_value("valu.json", dom, workload)
    valu_peak = 256 * 4 * 2.4e9 / 2.0  # wave64 VALU instr/s: 1024 SIMD-32s, 2 cycles each, 2.4 GHz
    pipeline_ms = sum(v for k, v in stage_ms.items() if k != "allreduce_exposed")
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
                               "forward+backward" + (f" + RCCL all-reduce of 56-B gradient rows ({args.reduce_chunks} chunks overlapping the chain)" if world > 1 else "")
                               + (" + one-rank RCCL rehearsal of the N > 1 step (all-reduce over a group of 1)" if args.rccl_single_rank else ""),
                   "gaussians": n, "width": w, "height": h, "views_per_step": world,
                   "pairs_per_view": p, "parallelism": f"views sharded dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "alg_bytes_per_launch": dom_bytes,
                     "avg_launch_ms": dom_ms,
                     "alg_bytes_walked": dom_walked, "achieved_walked": achieved_walked,
                     "frac_walked": achieved_walked / HBM_PEAK_GBS if achieved_walked else None,
                     "note": "achieved/frac: SURVEY.md §8d bytes (40 B per pair for all P pairs); _walked: the same "
                             "formula over the list entries the kernel walked (work counters, GsFrameStats)"},
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
        "work": walked,
        "launch": "eager" if graph is None else "hip_graph",
    }
    if comm is not None:
        result["comm"] = comm
        result["comm_gbs"] = comm["bus_gbs"]
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.rccl_single_rank:
        cp = device_copy_gbs(L, local_dev)
        result["hbm_copy_gbs"] = cp["best_gbs"]
        result["hbm_copy"] = cp
        result["cpu_baseline"] = cpu_baseline(args.cpu_threads or host_cpus()["threads"])
    if rank == 0:
        print(json.dumps(result), flush=True)
    rast.close()
    if split:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
