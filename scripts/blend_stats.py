"""Diagnostics (libgs_stats.so = -DGS_BLEND_STATS build): work counters of the forward and backward
blend kernels on the bench frame (1M Gaussians, 1080p, rig view 0), one frame."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from gaussiansplatting_amd import _lib, scene
from gaussiansplatting_amd.rasterizer import TiledRasterizer
n, w, h = 1_000_000, 1920, 1080
g = scene.synthetic_gaussians(n, 3, w, h)
u = scene.rig_uniforms(0, w, h)
gt = scene.synthetic_ground_truth(3, 0, w, h)
dev = torch.device("cuda:0")
dg = torch.from_numpy(g).to(dev)
dgt = torch.from_numpy(gt.view(np.int32)).to(dev)
out = torch.empty((h, w), dtype=torch.int32, device=dev)
grad = torch.empty((n, 28), dtype=torch.float32, device=dev)
r = TiledRasterizer(n, 0, w, h)
r.reserve_pairs(n * 256)
L = _lib.lib()
buf = np.zeros(32, dtype=np.uint64)
r.forward(dg, u, out)
r.backward(dg, grad, u, out, dgt)
torch.cuda.synchronize()
L.gs_debug_blend_stats(ctypes.c_void_p(buf.ctypes.data), 1)
r.forward(dg, u, out)
r.backward(dg, grad, u, out, dgt)
torch.cuda.synchronize()
assert L.gs_debug_blend_stats(ctypes.c_void_p(buf.ctypes.data), 1) == 0
P = r.num_pairs()
f, b = buf[:16].astype(float), buf[16:].astype(float)
print(f"P = {P}")
print(f"forward: waves {f[0]:.0f}, chunk steps {f[6]:.0f}, entries walked {f[1]:.0f} ({f[1]/P:.2f} per pair x4 waves), "
      f"selected {f[2]:.0f} ({f[2]/f[1]:.3f} of walked), pair steps {f[3]:.0f}, passing range ballot {f[4]:.0f} "
      f"({f[4]/max(1,f[3]):.3f}), contributing lanes / (2*64*passing) {f[5]/max(1,128*f[4]):.3f}")
print(f"backward: waves {b[0]:.0f}, chunks {b[10]:.0f}, entries walked {b[1]:.0f}, selected {b[2]:.0f} "
      f"({b[2]/max(1,b[1]):.3f}), beyond-end slots {b[3]:.0f}, pairs {b[8]:.0f}, pairs with no eval {b[9]:.0f} "
      f"({b[9]/max(1,b[8]):.3f})")
print(f"   band evals attempted {b[4]:.0f} ({b[4]/max(1,b[2]):.2f} per selected entry), passing ballot {b[5]:.0f} "
      f"({b[5]/max(1,b[4]):.3f}), in-range lanes / 64 {b[6]/max(1,64*b[5]):.3f}, contributing lanes / 64 {b[7]/max(1,64*b[5]):.3f}")
print("raw", buf.tolist())
r.close()
