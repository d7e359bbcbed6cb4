"""Diagnostics: does the forward blend's record gather at config-5 sizes depend on where the walked
Gaussians sit in memory? The same 5.2M-Gaussian frame rendered with the Gaussians in their generated
(random) order and permuted into camera-depth order (then the few hundred nearest Gaussians every tile
walks before saturating are neighbours in the record array). Run under rocprofv3 --kernel-trace and
compare forward_quad_kernel; argv[1] = "gid" | "depth"."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from gaussiansplatting_amd import scene
from gaussiansplatting_amd.rasterizer import TiledRasterizer

w, h, n = 1920, 1080, 5_200_000
g = scene.synthetic_gaussians(n, 5, w, h)
g[:, 4:7] += 1.2  # larger splats: lists of several thousand entries per tile, as config 5
if sys.argv[1] == "depth":
    g = g[np.argsort(g[:, 2], kind="stable")]
u = scene.make_uniforms(w, h)
dev = torch.device("cuda:0")
dg = torch.from_numpy(np.ascontiguousarray(g)).to(dev)
out = torch.empty((h, w), dtype=torch.int32, device=dev)
r = TiledRasterizer(n, 0, w, h)
r.reserve_pairs(200_000_000)
r.set_depth_sort(1)
for _ in range(8):
    r.forward(dg, u, out)
torch.cuda.synchronize()
st = r.frame_stats()
print(sys.argv[1], "pairs", r.num_pairs(), "fwd_walked", st["fwd_walked_entries"], flush=True)
r.close()
