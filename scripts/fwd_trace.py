"""Diagnostics (libgs_btrace.so = -DGS_BLEND_TRACE build): the forward blend's per-workgroup
start/end on the bench frame (wave 0 of each workgroup): span, the balanced span (sum of durations /
resident slots) and the residency over time."""
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
for _ in range(4):
    r.forward(dg, u, out)
    r.backward(dg, grad, u, out, dgt)
torch.cuda.synchronize()
L = _lib.lib()
buf = np.zeros((2, 16384, 2), dtype=np.uint64)
hw = np.zeros((2, 16384), dtype=np.uint32)
assert L.gs_debug_blend_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(hw.ctypes.data),
                              ctypes.c_size_t(buf.nbytes)) == 0
T = 8160
t = buf[0, :T].astype(np.int64)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
dur = en - st
span = en.max()
slots = 256 * 8  # workgroups of 4 waves resident at 8 waves per SIMD
print(f"forward span {span:.1f} us, workgroups {T}, sum(dur) {dur.sum():.0f} us, balanced {dur.sum() / slots:.1f} us, "
      f"mean {dur.mean():.1f}, max {dur.max():.1f}")
bins = np.arange(0, span + 10, 10)
print("  resident every 10 us:", [int(((st <= b) & (en > b)).sum()) for b in bins])
dec = np.array_split(np.arange(T), 10)
print("  dur by launch decile (mean, max):", [(round(float(dur[d].mean()), 1), round(float(dur[d].max()), 1)) for d in dec])
print("  start by launch decile (min, max):", [(round(float(st[d].min()), 1), round(float(st[d].max()), 1)) for d in dec])
b = buf[1, :2 * T].astype(np.int64)
b = b[b[:, 0] > 0]
bs, be = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0
print(f"  backward: first start {bs.min():.1f} us, last end {be.max():.1f} us, span {be.max() - bs.min():.1f}")
