"""Summary of scripts/ab.sh: per variant and repetition the step time and the stage times, then the
per-variant means; config lines and rocprofv3 kernel averages when present."""
import collections
import csv
import glob
import json
import os

O = "gpurun_out/ab"
per = collections.defaultdict(list)
for f in sorted(glob.glob(f"{O}/bench_*.log")):
    name = os.path.basename(f)[6:-4]
    var = name.rsplit("_", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            per[var].append(d)
            print(name, round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["stage_ms"].items()})
for var, runs in per.items():
    keys = runs[0]["stage_ms"].keys()
    mean = {k: round(sum(r["stage_ms"].get(k, 0.0) for r in runs) / len(runs), 4) for k in keys}
    print("MEAN", var, round(sum(r["ms_per_step"] for r in runs) / len(runs), 4), mean)
for f in sorted(glob.glob(f"{O}/cfg*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            print(os.path.basename(f)[:-4], round(d.get("ms_per_step", 0.0), 4),
                  {k: round(v, 4) for k, v in d.get("stage_ms", {}).items()})
for f in sorted(glob.glob(f"{O}/prof_*/**/*kernel_stats.csv", recursive=True)):
    print("PROF", f)
    with open(f) as fh:
        rows = list(csv.DictReader(fh))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
        print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.2f} us")
