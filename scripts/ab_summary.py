import glob, json, os
for f in sorted(glob.glob("gpurun_out/ab/bench_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(os.path.basename(f)[6:-4], round(d["ms_per_step"], 4),
                  {k: round(v, 4) for k, v in d["stage_ms"].items() })
