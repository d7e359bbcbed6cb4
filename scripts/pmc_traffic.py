"""Per-launch HBM traffic of every pipeline kernel from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE), corrected as MI355X_MICROARCH.md "HBM" prescribes: both counters are KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled. Each kernel is set
against its algorithmic (compulsory) bytes per launch, so the ratio says how much of
its traffic is re-reads or partial-line writes. Writes profiles/traffic.json ({workload: {stage:
bytes per launch, stage_read, stage_write, stage_alg, stage_ratio}}) for bench.py's roofline.traffic.

  python scripts/pmc_traffic.py PMC_DIR WORKLOAD N P W H [KERNEL_STATS_CSV]
  e.g. python scripts/pmc_traffic.py gpurun_out/round/pmc 1000000g_1920x1080 1000000 4651618 1920 1080 \
           gpurun_out/round/prof/bench_kernel_stats.csv

Every gs:: kernel that appears in the PMC passes or in the kernel-stats CSV must have an entry in
ALG below: the script fails otherwise, so a new kernel cannot silently drop out of the evidence.
"""
import collections
import csv
import json
import os
import sys

# kernel -> (stage name, algorithmic bytes per launch as a function of N, P, Npix, T). None: the
# kernel's compulsory bytes depend on data the script does not see (reported without a ratio).
ALG = {
    # projectGaussians: 56 B read per Gaussian, raster record + count + depth key + rect written
    "project_kernel": ("project", lambda n, p, npx, t: 132 * n),
    # per-tile depth order: the rect histogram reads each Gaussian's rect and count, writes [256][T]
    "tile_hist_rect_kernel": ("tile_hist", lambda n, p, npx, t: 20 * n + 4 * 256 * t),
    "tile_hist_kernel": ("tile_hist", lambda n, p, npx, t: 4 * p + 4 * 256 * t),
    "tile_colscan_kernel": ("tile_colscan", lambda n, p, npx, t: 8 * 256 * t),
    "tile_finish_kernel": ("tile_finish", lambda n, p, npx, t: 16 * 16 * t + 32 * t),
    # the gid walk: rects + counts read, the 4-B values written once, goff + slot fields
    "tile_scatter_gid_kernel": ("tile_scatter", lambda n, p, npx, t: 20 * n + 4 * p + 8 * n),
    "tile_scatter_kernel": ("tile_scatter", lambda n, p, npx, t: 8 * p + 4 * p),
    # every list read and written once, one 4-B depth key gathered per entry
    "tile_depth_sort_wave_kernel": ("depth_sort", lambda n, p, npx, t: 12 * p),
    "tile_seg_sort_kernel": ("depth_sort_jobs", None),  # (the long lists' entries: not known here)
    "tile_depth_sort_kernel": ("depth_sort_long", None),  # (round 4's long-list kernel)
    "tile_long_sort_kernel": ("depth_sort_long", None),  # (lists past the forward's in-LDS sort)
    "tile_reorder_kernel": ("tile_reorder", lambda n, p, npx, t: 12 * t),
    "tile_order_kernel": ("tile_order", lambda n, p, npx, t: 12 * t),
    "onesweep_kernel": ("depth_onesweep", lambda n, p, npx, t: 16 * n),
    "offsets_scan_kernel": ("offset_scan", lambda n, p, npx, t: 16 * n),
    "emit_slots_kernel": ("pair_emit", lambda n, p, npx, t: 24 * n + 8 * p),
    "radix_hist_kernel": ("radix_hist", lambda n, p, npx, t: 6 * p),
    "radix_scatter_kernel": ("radix_scatter", lambda n, p, npx, t: 12 * p),
    "chunk_base_kernel": ("chunk_base", lambda n, p, npx, t: 16 * t),
    "ranges_search_kernel": ("tile_ranges", lambda n, p, npx, t: 8 * t),
    # blend forward 40 P + 8 T + 8 Npix, backward 40 P + 8 T + 12 Npix
    "forward_kernel": ("forward_blend", lambda n, p, npx, t: 40 * p + 8 * t + 8 * npx),
    "backward_kernel": ("backward_blend", lambda n, p, npx, t: 40 * p + 8 * t + 12 * npx),
    # the per-Gaussian chain: 68 B of constants read, 64 B of gradients written
    "chain_kernel": ("chain", lambda n, p, npx, t: 68 * n + 64 * n),
    "chain_compact_kernel": ("chain", lambda n, p, npx, t: 68 * n + 64 * n),
    "forward_quad_kernel": ("forward_blend", lambda n, p, npx, t: 40 * p + 8 * t + 8 * npx),
    "emit_gid_kernel": ("pair_emit", lambda n, p, npx, t: 24 * n + 8 * p),
    "ranges_kernel": ("tile_ranges", lambda n, p, npx, t: 4 * p + 8 * t),
    "radix_digit_scan_kernel": ("radix_scan", None),
    "scan_reduce_kernel": ("scan", None), "scan_block_sums_kernel": ("scan", None),
    "scan_final_kernel": ("scan", None), "window_starts_kernel": ("pair_emit", None),
    # training-step kernels of config 5 (bench_configs.py): the rows path
    "unpack_kernel": ("unpack", lambda n, p, npx, t: 64 * n + 112 * n),
    "density_accumulate_kernel": ("density_accumulate", lambda n, p, npx, t: 20 * n + 2 * 24 * n),
    "density_accumulate_rows_kernel": ("density_accumulate", lambda n, p, npx, t: 20 * n + 2 * 24 * n),
    "density_mark_kernel": ("density_apply", None), "density_flag_kernel": ("density_apply", None),
    "density_demote_kernel": ("density_apply", None), "density_slots_kernel": ("density_apply", None),
    "density_emit_kernel": ("density_apply", None),
    # Adam: the Gaussian in and out, the 56-B gradient row, both 96-B moments in and out
    "adam_kernel": ("adam", lambda n, p, npx, t: 2 * 112 * n + 56 * n + 4 * 96 * n),
    "adam_follow_kernel": ("adam_follow", None), "adam_zero_kernel": ("adam_zero", None),
    "opacity_reset_kernel": ("opacity_reset", lambda n, p, npx, t: 8 * n),
    # loss: both RGBA8 images read, the per-tile partial sums written
    "loss_kernel": ("loss", lambda n, p, npx, t: 8 * npx), "loss_final_kernel": ("loss", None),
    "debug_pairs_kernel": ("debug", None), "debug_ranges_kernel": ("debug", None),
    "half_exp_check_kernel": ("debug", None), "float_exp_check_kernel": ("debug", None),
}


def kernel_key(raw: str) -> str:
    return raw.split("(")[0].replace("void ", "").replace("gs::", "").split("<")[0].strip().strip('"')


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[(kernel_key(r["Kernel_Name"]), r["Kernel_Name"].startswith(("gs::", "void gs::")))].append(
            float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def stats_kernels(path):
    out = set()
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        if name.startswith(("gs::", "void gs::")):
            out.add(kernel_key(name))
    return out


def main():
    if len(sys.argv) < 7:
        print(__doc__)
        return 2
    d, workload = sys.argv[1], sys.argv[2]
    n, p, w, h = (int(x) for x in sys.argv[3:7])
    npix, tiles = w * h, ((w + 15) // 16) * ((h + 15) // 16)
    fetch = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    ours = {k for (k, is_gs) in list(fetch) + list(write) if is_gs}
    if len(sys.argv) > 7:
        ours |= stats_kernels(sys.argv[7])
    missing = sorted(k for k in ours if k not in ALG)
    if missing:
        print(f"error: kernels without a stage / algorithmic bytes in ALG: {missing}", file=sys.stderr)
        return 1
    out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    try:
        allw = json.load(open(out_path))
    except Exception:
        allw = {}
    entry = {"_note": "bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), rocprofv3 PMC; "
                      "_alg = algorithmic bytes per launch (DESIGN.md §2), _ratio = measured / alg",
             "_sizes": {"gaussians": n, "pairs": p, "pixels": npix, "tiles": tiles}}
    for k in sorted(ours):
        stage, alg = ALG[k]
        fk, wk = fetch.get((k, True)), write.get((k, True))
        if fk is None or wk is None:
            print(f"error: kernel {k} missing from a PMC pass", file=sys.stderr)
            return 1
        key = stage if stage not in entry else f"{stage}:{k}"
        entry[key] = 2.0 * fk + wk
        entry[key + "_read"] = 2.0 * fk
        entry[key + "_write"] = wk
        entry[key + "_kernel"] = k
        if alg is not None:
            a = float(alg(n, p, npix, tiles))
            entry[key + "_alg"] = a
            entry[key + "_ratio"] = (2.0 * fk + wk) / a
    allw[workload] = entry
    json.dump(allw, open(out_path, "w"), indent=1, sort_keys=True)
    print(f"{'stage':22s} {'kernel':30s} {'read MB':>9s} {'write MB':>9s} {'total MB':>9s} {'alg MB':>9s} {'ratio':>6s}")
    for key in sorted(k for k in entry if k + "_kernel" in entry):
        alg = entry.get(key + "_alg")
        print(f"{key:22s} {entry[key + '_kernel']:30s} {entry[key + '_read'] / 1e6:9.1f} "
              f"{entry[key + '_write'] / 1e6:9.1f} {entry[key] / 1e6:9.1f} "
              f"{(alg or 0) / 1e6:9.1f} {entry.get(key + '_ratio', float('nan')):6.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
