"""Summarise rocprofv3 counter_collection CSVs per kernel (mean per dispatch)."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[name] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
    for k, d in agg.items():
        if "gs::" not in k:
            continue
        print(k, "vgpr/sgpr/lds", meta[k])
        print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
