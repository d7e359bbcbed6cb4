"""Diagnostics (libgs_ostrace.so = GS_OS_TRACE build): per-block phase timestamps of the sweep
kernels (depth histogram + slot scan, four depth passes, offsets scan) on the bench frame, or on n
Gaussians (argv[1], e.g. 5200000 for config 5's population)."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from gaussiansplatting_amd import _lib, scene
from gaussiansplatting_amd.rasterizer import TiledRasterizer
n, w, h = (int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000), 1920, 1080
g = scene.synthetic_gaussians(n, 3, w, h)
u = scene.rig_uniforms(0, w, h)
dev = torch.device("cuda:0")
dg = torch.from_numpy(g).to(dev)
out = torch.empty((h, w), dtype=torch.int32, device=dev)
r = TiledRasterizer(n, 0, w, h)
r.reserve_pairs(n * 256)
for _ in range(5):
    r.forward(dg, u, out)
torch.cuda.synchronize()
L = _lib.lib()
buf = np.zeros((6, 4096, 4), dtype=np.uint64)
assert L.gs_debug_os_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(buf.nbytes)) == 0
names = ["(unused)", "pass0", "pass1", "pass2", "pass3", "offsets"]
def os_items(m):  # gs_sort.hip
    if m <= 1 << 21:
        return 4
    cost = {it: -(-(-(-m // (1024 * it))) // 256) * it for it in (8, 10, 12)}
    return min(cost, key=lambda it: (cost[it], it))
tile = 1024 * os_items(n)
parts = {0: (n + tile - 1) // tile, 1: (n + tile - 1) // tile, 5: (n + 4095) // 4096}
for k in range(1, 6):
    m = parts.get(k, parts[1])
    t = buf[k, :m].astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # wall_clock64: 100 MHz
    print(f"{names[k]:11s} blocks {m}: start spread {us[:,0].max():6.2f} us | "
          f"p1-p0 mean {np.mean(us[:,1]-us[:,0]):6.2f} max {np.max(us[:,1]-us[:,0]):6.2f} | "
          f"p2-p1 mean {np.mean(us[:,2]-us[:,1]):6.2f} max {np.max(us[:,2]-us[:,1]):6.2f} | "
          f"p3-p2 mean {np.mean(us[:,3]-us[:,2]):6.2f} max {np.max(us[:,3]-us[:,2]):6.2f} | last end {us[:,3].max():6.2f}")
    # block order vs wait: correlation of ticket with p2-p1
    wait = us[:, 2] - us[:, 1]
    print("    wait by ticket decile:", np.round([wait[i * m // 10:(i + 1) * m // 10].mean() for i in range(10)], 2))
