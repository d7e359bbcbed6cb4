"""Diagnostic: where do non-finite gradients differ between the HIP path and the oracle in
test_edge_cases_mix's scene?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gaussiansplatting_amd import scene
from tests._helpers import run_gpu
from oracle import oracle as o

w, h = 256, 256
g = scene.synthetic_gaussians(4000, 21, w, h)
rng = np.random.default_rng(5)
idx = rng.choice(4000, 400, replace=False)
g[idx[:40], 0] = np.nan
g[idx[40:80], 1] = 2e6
g[idx[80:120], 8:12] = 0.0
g[idx[120:160], 4:7] = 3.0
g[idx[160:200], 4:7] = 8.0
g[idx[200:240], 4] = -9.0
g[idx[240:280], 12] = 20.0
g[idx[280:320], 12] = -9.0
g[idx[320:360], 13] = 5.0
g[idx[360:400], 13] = -5.0
u = scene.make_uniforms(w, h)
gt = scene.synthetic_ground_truth(21, 0, w, h)
ref = o.forward(g, u, w, h)
gpu = run_gpu(g, u, w, h, gt=gt)
gr, ab, nz = o.backward(g, ref, ref.rgba8, gt)
mine = gpu["grad"]
a, b = ~np.isfinite(gr), ~np.isfinite(mine)
rows = np.nonzero((a != b).any(1))[0]
print("rows differing:", len(rows), "ref nonfinite rows", int(a.any(1).sum()), "gpu nonfinite rows", int(b.any(1).sum()))
groups = {"nan_x": idx[:40], "y2e6": idx[40:80], "zeroq": idx[80:120], "huge": idx[120:160], "clamp": idx[160:200],
          "aniso": idx[200:240], "op20": idx[240:280], "opneg": idx[280:320], "c5": idx[320:360], "cm5": idx[360:400]}
for r in rows[:20]:
    grp = [k for k, v in groups.items() if r in v]
    cols = np.nonzero(a[r] != b[r])[0]
    print(r, grp, "cols", cols.tolist(), "ref", gr[r, cols].tolist(), "gpu", mine[r, cols].tolist())
    print("   input", g[r].tolist()[:16])
