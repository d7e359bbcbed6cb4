"""Summary of scripts/ab_cfg5.sh: per variant the config-5 step times and, from its kernel trace, each
kernel's time per frame over the last 4 frames (frames start at project_kernel)."""
import collections
import csv
import glob
import json
import sys

out, variants = sys.argv[1], sys.argv[2:]
per = {}
for v in variants:
    ms = []
    for f in sorted(glob.glob(f"{out}/cfg5_{v}_*.log")):
        ms.append(json.loads(open(f).read().strip().splitlines()[-1])["ms_per_step"])
    print(f"{v:12s} step ms " + " ".join(f"{x:.4f}" for x in ms))
    rows = list(csv.DictReader(open(glob.glob(f"{out}/prof_{v}/**/run_kernel_trace.csv", recursive=True)[0])))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] for r in rows]
    starts = [i for i, n in enumerate(names) if n.endswith("project_kernel")]
    F = min(4, len(starts))
    acc = collections.defaultdict(float)
    for r, n in zip(rows[starts[-F]:], names[starts[-F]:]):
        acc[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / F
    per[v] = acc
keys = sorted(set().union(*[set(a) for a in per.values()]), key=lambda k: -per[variants[0]].get(k, 0.0))
print(f"{'kernel (us per frame)':40s} " + " ".join(f"{v:>12s}" for v in variants))
for k in keys:
    print(f"{k[:40]:40s} " + " ".join(f"{per[v].get(k, 0.0):12.1f}" for v in variants))
print(f"{'total':40s} " + " ".join(f"{sum(per[v].values()):12.1f}" for v in variants))
