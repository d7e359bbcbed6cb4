"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (scripts/ab.sh PMC=...): per dispatch means,
and the issue-efficiency ratios (quad-cycle counters: WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY, MI355X_MICROARCH.md's PMC table)."""
import collections
import csv
import glob
import sys

O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
KERNELS = ("forward_kernel", "backward_kernel", "chain_kernel", "project_kernel", "tile_depth_sort_wave",
           "tile_scatter_gid", "tile_hist_gid", "offsets_scan")
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"{O}/pmc_*SQ*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = next((x for x in KERNELS if x in r["Kernel_Name"]), None)
        if k is None:
            continue
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
for k in KERNELS:
    if k not in vals:
        continue
    m = {c: vals[k][c] / max(1, len(disp[k][c])) for c in vals[k]}
    print(k)
    for c in sorted(m):
        print(f"  {c:24s} {m[c]:16.0f}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in m:
                print(f"  {c + ' / WAVE_CYCLES':40s} {m[c] / wc:6.3f}")
    if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVES" in m:
        print(f"  {'VALU insts per wave':40s} {m.get('SQ_INSTS_VALU', 0) / m['SQ_WAVES']:8.0f}")
