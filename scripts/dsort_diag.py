"""Round 3 diagnostic: pair count of the synthetic rig scene at several sizes through the library
named by GS_MI355X_LIB (compare libraries run by run)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from gaussiansplatting_amd import scene  # noqa: E402
from gaussiansplatting_amd.rasterizer import TiledRasterizer  # noqa: E402

W, H = 1920, 1080
dev = torch.device("cuda:0")
for n in [int(x) for x in sys.argv[1:]]:
    g = scene.synthetic_gaussians(n, 5, W, H)
    u = scene.rig_uniforms(0, W, H)
    r = TiledRasterizer(n, 0, W, H)
    r.reserve_pairs(80_000_000)
    r.set_tile_sort_path(1)
    dg = torch.from_numpy(g).to(dev)
    out = torch.zeros((H, W), dtype=torch.int32, device=dev)
    res = []
    for rep in range(2):
        r.forward(dg, u, out)
        torch.cuda.synchronize()
        res.append((r.num_pairs(), int(out.sum().item()), r.frame_stats()["scan_errors"]))
    print(os.environ.get("GS_MI355X_LIB", "default"), n, res, flush=True)
    r.close()
