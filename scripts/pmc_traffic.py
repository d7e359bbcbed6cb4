"""Per-launch HBM traffic of each pipeline kernel from two rocprofv3 PMC passes (FETCH_SIZE,
WRITE_SIZE), corrected as MI355X_MICROARCH.md "HBM" prescribes: both counters are KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide streaming read, so it is doubled. Writes
profiles/traffic.json ({workload: {stage: bytes per launch}}) for bench.py's roofline.traffic.

  python scripts/pmc_traffic.py gpurun_out/pmc 1000000g_1920x1080
"""
import collections
import csv
import json
import os
import sys

STAGE_OF = {"project_kernel": "project", "emit_kernel": "pair_emit", "emit_slots_kernel": "pair_emit",
            "ranges_kernel": "tile_ranges", "tile_hist_kernel": "tile_hist",
            "tile_scatter_kernel": "tile_scatter", "tile_colscan_kernel": "tile_colscan",
            "forward_kernel": "forward_blend", "backward_kernel": "backward_blend",
            "chain_kernel": "chain", "radix_scatter_kernel": "radix_scatter",
            "radix_hist_kernel": "radix_hist", "tile_order_kernel": "tile_order",
            "onesweep_kernel": "depth_onesweep",
            "offsets_scan_kernel": "offset_scan", "tile_finish_kernel": "tile_finish",
            "strip_sort_kernel": "strip_sort"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gs::", "").split("<")[0]
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d, workload = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    try:
        allw = json.load(open(out_path))
    except Exception:
        allw = {}
    entry = {"_note": "bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), rocprofv3 PMC"}
    for k, stage in STAGE_OF.items():
        if k in fetch and k in write:
            entry[stage] = 2.0 * fetch[k] + write[k]
            entry[stage + "_read"] = 2.0 * fetch[k]
            entry[stage + "_write"] = write[k]
    allw[workload] = entry
    json.dump(allw, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in sorted(entry.items()):
        if not k.startswith("_"):
            print(f"{k:28s} {v/1e6:10.1f} MB")


if __name__ == "__main__":
    main()
