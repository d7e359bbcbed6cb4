"""Issue efficiency per kernel from rocprofv3 --pmc counter_collection CSVs (any number of passes, e.g.
gpurun_out/sq/run_counter_collection.csv gpurun_out/sq2/...): per-dispatch means and the fractions of
SQ_WAVE_CYCLES (quad-cycle counters: WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, per
MI355X_MICROARCH.md's PMC table), VALU instructions per wave."""
import collections
import csv
import sys

KERNELS = ("forward_quad_kernel", "backward_kernel", "chain_kernel", "chain_screen_kernel", "chain_list_kernel",
           "project_kernel", "tile_scatter_gid", "tile_hist_rect", "offsets_scan", "emit_slots_kernel", "onesweep_kernel",
           "radix_hist_kernel", "radix_scatter_kernel", "loss_kernel", "tile_long_sort_kernel")
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        k = next((x for x in KERNELS if x in r["Kernel_Name"]), None)
        if k is None:
            continue
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k in KERNELS:
    if k not in vals:
        continue
    m = {c: vals[k][c] / max(1, len(disp[k][c])) for c in vals[k]}
    wc = m.get("SQ_WAVE_CYCLES")
    parts = []
    if wc:
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS"):
            if c in m:
                parts.append(f"{c[3:].lower()} {m[c] / wc:.3f}")
    if m.get("SQ_WAVES") and "SQ_INSTS_VALU" in m:
        parts.append(f"valu/wave {m['SQ_INSTS_VALU'] / m['SQ_WAVES']:.0f}")
        parts.append(f"valu insts {m['SQ_INSTS_VALU']:.3e}")
    print(f"{k:22s} " + ", ".join(parts))
