"""Round 3 diagnostic: per-Gaussian pair counts and depth keys of one frame of the synthetic rig
scene through the library named by GS_MI355X_LIB, saved for an offline comparison."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussiansplatting_amd import scene  # noqa: E402
from gaussiansplatting_amd.rasterizer import TiledRasterizer  # noqa: E402

W, H = 1920, 1080
dev = torch.device("cuda:0")
n = int(sys.argv[1])
g = scene.synthetic_gaussians(n, 5, W, H)
u = scene.rig_uniforms(0, W, H)
r = TiledRasterizer(n, 0, W, H)
r.reserve_pairs(80_000_000)
r.set_tile_sort_path(1)
dg = torch.from_numpy(g).to(dev)
out = torch.zeros((H, W), dtype=torch.int32, device=dev)
r.forward(dg, u, out)
torch.cuda.synchronize()
keys, vals = r.sorted_pairs()
cnt = np.bincount(vals, minlength=n).astype(np.uint16)
dk = np.zeros(n, dtype=np.uint32)
dk[vals] = (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)
tag = os.path.basename(os.environ.get("GS_MI355X_LIB", "default")).replace(".so", "")
os.makedirs("gpurun_out/dd", exist_ok=True)
np.savez_compressed(f"gpurun_out/dd/{tag}_{n}.npz", cnt=cnt, dk=dk)
print(tag, n, r.num_pairs(), flush=True)
