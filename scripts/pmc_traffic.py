"""Per-launch HBM traffic of every pipeline kernel from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE), corrected as MI355X_MICROARCH.md "HBM" prescribes: both counters are KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled. Each kernel is set
against its algorithmic (compulsory) bytes per launch, so the ratio says how much
of its traffic is re-reads or partial-line writes. Writes profiles/traffic.json ({workload: {stage:
bytes per launch, stage_read, stage_write, stage_alg, stage_ratio}}) for bench.py's roofline.traffic.

  python scripts/pmc_traffic.py PMC_DIR WORKLOAD N P W H [KERNEL_STATS_CSV] [--facts BENCH_LOG]
  e.g. python scripts/pmc_traffic.py gpurun_out/round/pmc 1000000g_1920x1080 1000000 4651618 1920 1080 \
           gpurun_out/round/prof/bench_kernel_stats.csv --facts gpurun_out/round/bench.log

--facts takes the bench line (bench.py or bench_configs.py) of the same workload: its "work" object
(GsFrameStats: the list entries the blends walked, the reached Gaussians and their slots) makes the
blends' and the chain's algorithmic bytes a compulsory count -- the blends stop at each pixel's last
contributor, so most of a deep list is never read and 40 B x P overstates them (config 5: 0.10-0.22 of
it measured) -- and config 5's density_apply record gives the apply's and the moment follow's counts.
Without facts the §8d formulas over all P pairs are used.

Every gs:: kernel that appears in the PMC passes or in the kernel-stats CSV must have an entry in
ALG below: the script fails otherwise, so a new kernel cannot silently drop out of the evidence.
"""
import collections
import csv
import json
import os
import sys


class Sizes:
    """The workload's counts: n Gaussians, p pairs, npx pixels, t tiles, and (facts) wf / wb the list
    entries the forward / backward walked, r the reached Gaussians, sr their slots, n_in / n_out /
    kept / pruned the last density apply's counts (config 5)."""

    def __init__(self, n, p, npx, t, facts=None):
        self.n, self.p, self.npx, self.t = n, p, npx, t
        work = (facts or {}).get("work") or {}
        self.wf = work.get("fwd_walked_entries") or p
        self.wb = work.get("bwd_walked_entries") or p
        self.r = work.get("reached_gaussians")
        self.sr = work.get("reached_slots")
        ap = ((facts or {}).get("config") or {}).get("density_apply") or {}
        self.n_in = ap.get("n_before")
        self.n_out = ap.get("n_after")
        self.pruned = ap.get("num_pruned", 0)
        self.split = ap.get("num_split", 0)
        self.cloned = ap.get("num_cloned", 0)


def _chain(c):
    """The plain / compacting chain into gradient rows or records: tile count + reached tag per
    Gaussian; for each reached one its 68 B of constants, its slot base and its slots (40 B each);
    one gradient row (56 B) per Gaussian written. Without facts: §8d's 68 + 64 B per Gaussian."""
    if c.r is None:
        return 68 * c.n + 64 * c.n
    return 5 * c.n + c.r * (68 + 4) + 40 * c.sr + 56 * c.n


def _fused(c):
    """gs_backward_step's chain -> density -> Adam: every Gaussian's count, reached tag and live flag
    and its 112-B record (Adam's clamps and renormalisation run on all of them); for each reached
    one its slot base and slots, its moments (the four live 16-B quads of each record) read and
    written, its record written back and its density statistics (20 B) read and written."""
    if c.r is None:
        return None
    return c.n * (4 + 1 + 1 + 112) + c.r * (4 + 2 * 2 * 64 + 112 + 2 * 20) + 40 * c.sr


def _split(step, list_part):
    """The compacting path's two launches (gs_chain.hip): chain_screen_kernel reads every Gaussian's
    count and reached tag (with kStep also its live flag and 112-B record: Adam's clamps run on all),
    stores the unreached ones' zero gradient rows (without kStep) and lists the others (4 B each);
    chain_list_kernel reads the list and, per reached Gaussian, its 68 B of constants, slot base and
    slots (40 B each), and writes its row, or with kStep reads and writes its moments (the four live
    quads of each record), record and density statistics (20 B)."""
    def f(c):
        if c.r is None:
            return None
        if not step:
            return 4 * c.r + c.r * (68 + 4) + 40 * c.sr + 56 * c.r if list_part else 5 * c.n + 56 * (c.n - c.r) + 4 * c.r
        if list_part:
            return 4 * c.r + c.r * (4 + 112 + 2 * 2 * 64 + 112 + 2 * 20) + 40 * c.sr
        return c.n * (4 + 1 + 1 + 112) + 4 * c.r
    return f


def _follow(c):
    """Adam moments following an apply: marker + offset per input Gaussian, the moments (2 x 96 B) of
    every kept / cloned original read, every output record written (+ its live byte)."""
    if c.n_in is None:
        return None
    return 8 * c.n_in + 192 * (c.n_in - c.pruned - c.split) + 193 * c.n_out


def _apply(per_in, per_out=0):
    return lambda c: None if c.n_in is None else per_in * c.n_in + per_out * c.n_out


# kernel -> (stage name, algorithmic bytes per launch as a function of the Sizes). None: the
# kernel's compulsory bytes depend on data the script does not see (reported without a ratio).
ALG = {
    # projectGaussians: 56 B read per Gaussian, raster record + count + depth key + rect written
    "project_kernel": ("project", lambda c: 132 * c.n),
    # per-tile depth order: the rect histogram reads each Gaussian's rect (8 B) and count, writes the
    # [256][T] slice counts and one count per 64-Gaussian chunk
    "tile_hist_rect_kernel": ("tile_hist", lambda c: 12 * c.n + 4 * 256 * c.t + c.n // 16),
    "tile_hist_kernel": ("tile_hist", lambda c: 4 * c.p + 4 * 256 * c.t),
    "tile_colscan_kernel": ("tile_colscan", lambda c: 8 * 256 * c.t),
    # the 16 chunk sums per tile read and written back as prefixes; ranges, launch order, chunk bases,
    # XCD groups and the zeroed work counters written
    "tile_finish_kernel": ("tile_finish", lambda c: 2 * 64 * c.t + 24 * c.t),
    # the gid walk: rects + counts read, the 4-B values written once, goff + slot fields
    "tile_scatter_gid_kernel": ("tile_scatter", lambda c: 20 * c.n + 4 * c.p + 8 * c.n),
    "tile_scatter_kernel": ("tile_scatter", lambda c: 8 * c.p + 4 * c.p),
    "tile_long_sort_kernel": ("depth_sort_long", None),  # (lists past the forward's in-LDS sort)
    "tile_reorder_kernel": ("tile_reorder", lambda c: 12 * c.t),
    "onesweep_kernel": ("depth_onesweep", lambda c: 16 * c.n),
    "offsets_scan_kernel": ("offset_scan", lambda c: 16 * c.n),
    "emit_slots_kernel": ("pair_emit", lambda c: 24 * c.n + 8 * c.p),
    # the two 8-bit-or-narrower LSD passes over u16 tile keys (T <= 65536): each histogram reads the
    # keys; the first scatter reads and writes key + value (12 B), the last writes no keys (10 B)
    "radix_hist_kernel": ("radix_hist", lambda c: 2 * c.p),
    "radix_scatter_kernel": ("radix_scatter", lambda c: 11 * c.p),
    "chunk_base_kernel": ("chunk_base", lambda c: 16 * c.t),
    "ranges_search_kernel": ("tile_ranges", lambda c: 8 * c.t),
    # blend forward 40 B per pair + 8 T + 8 Npix, backward 40 B per pair + 8 T + 12
    # Npix, over the pairs each walked (facts; all P without them)
    "forward_quad_kernel": ("forward_blend", lambda c: 40 * c.wf + 8 * c.t + 8 * c.npx),
    "backward_kernel": ("backward_blend", lambda c: 40 * c.wb + 8 * c.t + 12 * c.npx),
    "chain_kernel": ("chain", _chain),
    "chain_kernel<step>": ("fused_tail", _fused),
    "chain_screen_kernel": ("chain_screen", _split(False, False)),
    "chain_list_kernel": ("chain_list", _split(False, True)),
    "chain_screen_kernel<step>": ("fused_tail_screen", _split(True, False)),
    "chain_list_kernel<step>": ("fused_tail_list", _split(True, True)),
    "emit_gid_kernel": ("pair_emit", lambda c: 24 * c.n + 8 * c.p),
    "ranges_kernel": ("tile_ranges", lambda c: 4 * c.p + 8 * c.t),
    "radix_digit_scan_kernel": ("radix_scan", None),
    "scan_reduce_kernel": ("scan", None), "scan_block_sums_kernel": ("scan", None),
    "scan_final_kernel": ("scan", None),
    # training-step kernels of config 5 (bench_configs.py)
    "unpack_kernel": ("unpack", lambda c: 64 * c.n + 112 * c.n),
    "density_accumulate_kernel": ("density_accumulate", lambda c: 20 * c.n + 2 * 24 * c.n),
    "density_accumulate_rows_kernel": ("density_accumulate", lambda c: 20 * c.n + 2 * 24 * c.n),
    # the apply (once per 100 iterations): marks from the statistics (8 B) and the log-scale and raw
    # opacity (16 B read, the marker written), slots over the markers, the survivors emitted
    "density_mark_kernel": ("density_apply", _apply(4 + 4 + 16 + 4)),
    "density_slots_kernel": ("density_apply", _apply(8)),
    "density_flag_kernel": ("density_apply", None), "density_demote_kernel": ("density_apply", None),
    "density_emit_kernel": ("density_apply", _apply(8 + 112, 112)),
    # Adam: the Gaussian in and out, the 56-B gradient row, both 96-B moments in and out
    "adam_kernel": ("adam", lambda c: 2 * 112 * c.n + 56 * c.n + 4 * 96 * c.n),
    "adam_follow_kernel": ("adam_follow", _follow), "adam_zero_kernel": ("adam_zero", None),
    "opacity_reset_kernel": ("opacity_reset", lambda c: 8 * c.n),
    # loss: both RGBA8 images read, the per-tile partial sums written
    "loss_kernel": ("loss", lambda c: 8 * c.npx), "loss_final_kernel": ("loss", None),
    "debug_pairs_kernel": ("debug", None), "debug_ranges_kernel": ("debug", None),
    "half_exp_check_kernel": ("debug", None), "float_exp_check_kernel": ("debug", None),
    "copy_stream_kernel": ("hbm_copy", None),
}


def kernel_key(raw: str) -> str:
    name = raw.split("(")[0].replace("void ", "").replace("gs::", "").strip().strip('"')
    base = name.split("<")[0].strip()
    if base.startswith("chain_") and "<" in name:  # chain kernels <kStep>: the fused tail apart
        args = [a.strip() for a in name.split("<", 1)[1].rstrip(">").split(",")]
        if args and args[-1] in ("true", "1"):
            return base + "<step>"
    return base


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
    argv = list(sys.argv)
    facts = None
    if "--facts" in argv:
        i = argv.index("--facts")
        facts = json.loads(open(argv[i + 1]).read().strip().splitlines()[-1])
        del argv[i:i + 2]
    if len(argv) < 7:
        print(__doc__)
        return 2
    d, workload = argv[1], argv[2]
    n, p, w, h = (int(x) for x in argv[3:7])
    npix, tiles = w * h, ((w + 15) // 16) * ((h + 15) // 16)
    sizes = Sizes(n, p, npix, tiles, facts)
    fetch = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    ours = {k for (k, is_gs) in list(fetch) + list(write) if is_gs}
    if len(argv) > 7:
        ours |= stats_kernels(argv[7])
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
             "_sizes": {"gaussians": n, "pairs": p, "pixels": npix, "tiles": tiles,
                        "fwd_walked": sizes.wf, "bwd_walked": sizes.wb, "reached": sizes.r,
                        "reached_slots": sizes.sr}}
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
        a = alg(sizes) if alg is not None else None
        if a is not None:
            entry[key + "_alg"] = float(a)
            entry[key + "_ratio"] = (2.0 * fk + wk) / float(a)
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
