"""Diagnostics (libgs_btrace.so = -DGS_BLEND_TRACE build): the backward blend's per-wave start/end
on the bench frame, for a heavy-tile split setting (argv[1], -1 automatic, 0 off): the span, the
ideal balanced span (sum of wave durations / resident slots), and who is running in the tail."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from gaussiansplatting_amd import _lib, scene
from gaussiansplatting_amd.rasterizer import TiledRasterizer
split = int(sys.argv[1]) if len(sys.argv) > 1 else 0
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
r.set_backward_split(split)
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
H = 0 if split == 0 else (T if split < 0 else min(split, T))
G = T + H
t = buf[1, :G].astype(np.int64)
t0 = t[:, 0].min()
st, en = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
dur = en - st
span = en.max()
print(f"split {split} (H={H}): backward span {span:.1f} us, waves {G}, sum(dur) {dur.sum():.0f} us, "
      f"sum/4096 {dur.sum() / 4096:.1f} us, mean {dur.mean():.1f}, max {dur.max():.1f}")
bins = np.arange(0, span + 20, 20)
print("  resident every 20 us:", [int(((st <= b) & (en > b)).sum()) for b in bins])
for frac in (0.6, 0.75, 0.9):
    tb = frac * span
    alive = np.nonzero((st <= tb) & (en > tb))[0]
    print(f"  alive at {frac:.2f} span ({tb:.0f} us): {alive.size}; launch pos pct "
          f"{np.percentile(alive, [0, 25, 50, 75, 100]).round().tolist() if alive.size else []}; "
          f"their start median {np.median(st[alive]) if alive.size else 0:.0f} dur median {np.median(dur[alive]) if alive.size else 0:.0f}")
# duration by launch-position decile
dec = np.array_split(np.arange(G), 10)
print("  dur by launch decile (mean, max):", [(round(float(dur[d].mean()), 1), round(float(dur[d].max()), 1)) for d in dec])
print("  start by launch decile (min):", [round(float(st[d].min()), 1) for d in dec])
if False:
    a, b = dur[0:2 * H:2], dur[1:2 * H:2]
    print(f"  split halves: first mean {a.mean():.1f} max {a.max():.1f}; second mean {b.mean():.1f} max {b.max():.1f}")
if H:
    b, f = dur[:H], dur[H:2 * H]  # back parts, front quarters
    print(f"  back halves: mean {b.mean():.1f} max {b.max():.1f}; front halves: mean {f.mean():.1f} max {f.max():.1f}; "
          f"front start min {st[H:2 * H].min():.1f}; front wait (start - back end) min "
          f"{(st[H:2 * H] - en[:H]).min():.1f} us")
