"""VALU instructions per launch of each pipeline kernel from a rocprofv3 SQ counter pass
(SQ_INSTS_VALU: wave-level VALU instructions summed over the dispatch). Writes
profiles/valu.json ({workload: {stage: instructions per launch}}) for bench.py's roofline_valu.

  python scripts/sq_valu.py gpurun_out/sq/<...>/run_counter_collection.csv 1000000g_1920x1080
"""
import collections
import csv
import json
import os
import sys

STAGE_OF = {"forward_kernel": "forward_blend", "backward_kernel": "backward_blend",
            "chain_kernel": "chain", "project_kernel": "project", "emit_slots_kernel": "pair_emit"}


def main():
    path, workload = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "SQ_INSTS_VALU":
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gs::", "").split("<")[0]
        if name in STAGE_OF:
            acc[STAGE_OF[name]].append(float(r["Counter_Value"]))
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "valu.json")
    data = {}
    if os.path.exists(out_path):
        data = json.load(open(out_path))
    entry = {k: sum(v) / len(v) for k, v in acc.items()}
    entry["_note"] = "SQ_INSTS_VALU per launch (wave64 instructions), rocprofv3 PMC"
    data[workload] = entry
    json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in sorted(entry.items()):
        print(f"{k:20s} {v}")


if __name__ == "__main__":
    main()
