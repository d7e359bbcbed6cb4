"""Diagnostics (libgs_btrace.so = -DGS_BLEND_TRACE build): per-workgroup start/end timestamps of the
forward and backward blend kernels on the bench frame -> occupancy over time (tail analysis)."""
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
for k, name in ((0, "forward"), (1, "backward")):
    t = buf[k, :T].astype(np.int64)
    t0 = t[:, 0].min()
    st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # us (100 MHz)
    dur = en - st
    total = en.max()
    print(f"{name}: span {total:.1f} us, block dur mean {dur.mean():.1f} max {dur.max():.1f} us, "
          f"starts: last {st.max():.1f} us; sum(dur) {dur.sum():.0f} us")
    # resident workgroups over time (10 us bins)
    bins = np.arange(0, total + 10, 10)
    occ = [int(((st <= b) & (en > b)).sum()) for b in bins]
    print("   resident workgroups every 10 us:", occ)
    # longest blocks and their launch positions
    idx = np.argsort(dur)[::-1][:8]
    print("   longest:", [(int(i), round(float(dur[i]), 1), round(float(st[i]), 1)) for i in idx])
fd = (buf[0, :T, 1].astype(np.int64) - buf[0, :T, 0].astype(np.int64)) / 100.0
bd = (buf[1, :T, 1].astype(np.int64) - buf[1, :T, 0].astype(np.int64)) / 100.0
print("corr(forward block dur, backward block dur) by launch index:", np.corrcoef(fd, bd)[0, 1])
ranges = r.tile_ranges()
print("launch-order position of the 20 longest backward blocks:", np.argsort(bd)[::-1][:20].tolist())
# how good is launch order (list-length LPT) as a predictor of backward duration
from scipy.stats import spearmanr
print("spearman(launch index, backward dur):", spearmanr(np.arange(T), bd).correlation)
print("spearman(forward dur, backward dur):", spearmanr(fd, bd).correlation)
