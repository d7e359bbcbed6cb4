"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle/libgs_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The oracle is a CPU restatement of the reference's Metal kernels (see gs_oracle.h; parity
unpinned — the reference cannot run here).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_uint16, c_uint32, c_uint64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgs_oracle.so")
_lib = None


def use_library(path: str) -> None:
    """Load the oracle from another build of oracle/gs_oracle.c (bench.py's CPU baseline builds it
    -march=native for the host it runs on). Same source, same results."""
    global _lib, LIB_PATH
    LIB_PATH = path
    _lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make oracle/libgs_oracle.so`")
        L = ctypes.CDLL(LIB_PATH)
        L.gso_expf.restype = c_float
        L.gso_expf.argtypes = [c_float]
        L.gso_half.restype = c_float
        L.gso_half.argtypes = [c_float]
        L.gso_half_bits.restype = c_uint16
        L.gso_half_bits.argtypes = [c_float]
        L.gso_project.restype = None
        L.gso_project.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_int]
        L.gso_generate_pairs.restype = c_uint64
        L.gso_generate_pairs.argtypes = [c_void_p, c_uint32, c_uint32, c_uint64, c_void_p, c_void_p]
        L.gso_sort_pairs.restype = None
        L.gso_sort_pairs.argtypes = [c_void_p, c_void_p, c_uint64, c_int]
        L.gso_build_tile_ranges.restype = None
        L.gso_build_tile_ranges.argtypes = [c_void_p, c_uint64, c_uint32, c_void_p, c_int]
        L.gso_forward_blend.restype = None
        L.gso_forward_blend.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_uint32,
                                        c_uint32, c_void_p, c_void_p, c_void_p, c_int]
        L.gso_backward.restype = None
        L.gso_backward.argtypes = [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p,
                                   c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int]
        L.gso_backward_shadow.restype = None
        L.gso_backward_shadow.argtypes = L.gso_backward.argtypes[:12] + [c_void_p, c_int]
        L.gso_backward_full.restype = None
        L.gso_backward_full.argtypes = L.gso_backward.argtypes[:14] + [c_void_p, c_void_p, c_int]
        L.gso_forward.restype = c_uint64
        L.gso_forward.argtypes = [c_void_p, c_uint32, c_void_p, c_uint32, c_uint32, c_uint64,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_int]
        L.gso_density_accumulate.restype = None
        L.gso_density_accumulate.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]
        L.gso_density_apply.restype = c_uint64
        L.gso_density_apply.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p, c_uint64, c_float,
                                        c_float, c_float, c_float, c_uint64, c_uint64, c_void_p,
                                        c_void_p, c_void_p]
        L.gso_adam_step.restype = None
        L.gso_adam_step.argtypes = [c_void_p, c_void_p, c_uint32] + [c_void_p] * 11 + [c_float] * 5
        L.gso_opacity_reset.restype = None
        L.gso_opacity_reset.argtypes = [c_void_p, c_uint32, c_float]
        L.gso_loss.restype = c_double
        L.gso_loss.argtypes = [c_void_p, c_void_p, c_uint32, c_uint32, c_float, c_void_p, c_int]
        L.gso_density_uniform.restype = c_float
        L.gso_density_uniform.argtypes = [c_uint64, c_uint64, c_uint32]
        _lib = L
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def _u(uniforms: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(np.asarray(uniforms, dtype=np.float32).reshape(-1)).copy()
    assert u.size == 60
    return u


class ForwardResult:
    __slots__ = ("num_pairs", "projected", "keys", "values", "ranges", "last_idx", "rgba8",
                 "rgb", "uniforms", "w", "h")


def forward(gaussians: np.ndarray, uniforms: np.ndarray, w: int, h: int,
            max_pairs: int | None = None, threads: int = 8) -> ForwardResult:
    """Whole TiledRasterizer::forward (tiled_rasterizer.mm:275-672) on the CPU."""
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    tx, ty = (w + 15) // 16, (h + 15) // 16
    cap = int(max_pairs if max_pairs is not None else max(n * min(256, tx * ty), 1))
    u = _u(uniforms)
    uu = u.view(np.uint32)
    uu[56], uu[57], uu[58] = tx, ty, n
    r = ForwardResult()
    r.projected = np.zeros((max(n, 1), 22), dtype=np.float32)
    r.keys = np.zeros(max(cap, 1), dtype=np.uint64)
    r.values = np.zeros(max(cap, 1), dtype=np.uint32)
    r.ranges = np.zeros((tx * ty, 2), dtype=np.uint32)
    r.last_idx = np.zeros((h, w), dtype=np.uint32)
    r.rgba8 = np.zeros((h, w), dtype=np.uint32)
    r.rgb = np.zeros((h, w, 3), dtype=np.float32)
    p = lib().gso_forward(_p(g), n, _p(u), w, h, cap, _p(r.projected), _p(r.keys), _p(r.values),
                          _p(r.ranges), _p(r.last_idx), _p(r.rgba8), _p(r.rgb), threads)
    r.num_pairs = int(p)
    r.keys = r.keys[:p]
    r.values = r.values[:p]
    r.projected = r.projected[:n]
    r.uniforms = u
    r.w, r.h = w, h
    return r


def backward(gaussians: np.ndarray, fwd: ForwardResult, rendered: np.ndarray,
             ground_truth: np.ndarray, threads: int = 8, stats: bool = True):
    """tiledBackward (tiled_shaders.metal:388-738).

    Returns (grad, abs_terms, noise) as (N, 28) float64: the sum of the float per-pixel terms,
    the sum of their magnitudes, and the sum of |float term - fp64 term| (rounding noise)."""
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    grad = np.zeros((max(n, 1), 28), dtype=np.float64)
    absg = np.zeros((max(n, 1), 28), dtype=np.float64)
    noise = np.zeros((max(n, 1), 28), dtype=np.float64)
    vals = fwd.values if fwd.values.size else np.zeros(1, dtype=np.uint32)
    rend = np.ascontiguousarray(rendered, dtype=np.uint32)
    gt = np.ascontiguousarray(ground_truth, dtype=np.uint32)
    lib().gso_backward(_p(g), _p(fwd.projected if n else np.zeros((1, 22), np.float32)), n,
                       _p(vals), _p(fwd.ranges), _p(fwd.uniforms), fwd.w, fwd.h,
                       _p(fwd.last_idx), _p(rend), _p(gt), _p(grad),
                       _p(absg) if stats else None, _p(noise) if stats else None, threads)
    return grad[:n], absg[:n], noise[:n]


def backward_shadow(gaussians: np.ndarray, fwd: ForwardResult, rendered: np.ndarray,
                    ground_truth: np.ndarray, threads: int = 8):
    """(grad, shadow): backward()'s float sums and their fp64 shadow, every per-pixel term
    recomputed in double from the same float inputs. Where a float intermediate of the reference
    overflows (huge splats), grad is NaN and shadow is the finite value."""
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    grad = np.zeros((max(n, 1), 28), dtype=np.float64)
    shadow = np.zeros((max(n, 1), 28), dtype=np.float64)
    vals = fwd.values if fwd.values.size else np.zeros(1, dtype=np.uint32)
    rend = np.ascontiguousarray(rendered, dtype=np.uint32)
    gt = np.ascontiguousarray(ground_truth, dtype=np.uint32)
    lib().gso_backward_shadow(_p(g), _p(fwd.projected if n else np.zeros((1, 22), np.float32)), n,
                              _p(vals), _p(fwd.ranges), _p(fwd.uniforms), fwd.w, fwd.h,
                              _p(fwd.last_idx), _p(rend), _p(gt), _p(grad), _p(shadow), threads)
    return grad[:n], shadow[:n]


def backward_full(gaussians: np.ndarray, fwd: ForwardResult, rendered: np.ndarray,
                  ground_truth: np.ndarray, threads: int = 8):
    """backward() and backward_shadow() in one pass: (grad, abs_terms, noise, shadow, cond), each
    (N, 28) float64. `shadow` is the sum of the per-pixel terms recomputed in fp64 from the same
    float inputs: the value the reference's float sum approximates to within `noise` (the rounding
    error it happened to make). `cond` bounds the error any float evaluation of the same per-pixel
    steps may make (first-order conditioning; gs_oracle.c COND_EXP_REL)."""
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    outs = [np.zeros((max(n, 1), 28), dtype=np.float64) for _ in range(5)]
    vals = fwd.values if fwd.values.size else np.zeros(1, dtype=np.uint32)
    rend = np.ascontiguousarray(rendered, dtype=np.uint32)
    gt = np.ascontiguousarray(ground_truth, dtype=np.uint32)
    lib().gso_backward_full(_p(g), _p(fwd.projected if n else np.zeros((1, 22), np.float32)), n,
                            _p(vals), _p(fwd.ranges), _p(fwd.uniforms), fwd.w, fwd.h,
                            _p(fwd.last_idx), _p(rend), _p(gt), *[_p(o) for o in outs], threads)
    return tuple(o[:n] for o in outs)


def project(gaussians: np.ndarray, uniforms: np.ndarray, w: int, h: int,
            threads: int = 8) -> np.ndarray:
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    u = _u(uniforms)
    uu = u.view(np.uint32)
    uu[56], uu[57], uu[58] = (w + 15) // 16, (h + 15) // 16, n
    out = np.zeros((max(n, 1), 22), dtype=np.float32)
    lib().gso_project(_p(g), n, _p(u), _p(out), threads)
    return out[:n]


def sorted_pairs(gaussians: np.ndarray, uniforms: np.ndarray, w: int, h: int, threads: int = 8):
    """projectGaussians -> generateTilePairs -> 64-bit radix sort -> buildTileRanges only
    (tiled_rasterizer.mm:275-440), without the blend: for pair-heavy scenes.
    Returns (keys, values, ranges[T, 2])."""
    p = project(gaussians, uniforms, w, h, threads)
    n = p.shape[0]
    tx, ty = (w + 15) // 16, (h + 15) // 16
    L = lib()
    total = int(L.gso_generate_pairs(_p(p), n, tx, 0, None, None))
    keys = np.zeros(max(total, 1), dtype=np.uint64)
    vals = np.zeros(max(total, 1), dtype=np.uint32)
    got = int(L.gso_generate_pairs(_p(p), n, tx, total, _p(keys), _p(vals)))
    assert got == total
    keys, vals = keys[:total], vals[:total]
    L.gso_sort_pairs(_p(keys), _p(vals), total, threads)
    ranges = np.zeros((tx * ty, 2), dtype=np.uint32)
    L.gso_build_tile_ranges(_p(keys), total, tx * ty, _p(ranges), threads)
    return keys, vals, ranges


def sort_pairs(keys: np.ndarray, values: np.ndarray, threads: int = 8):
    k = np.ascontiguousarray(keys, dtype=np.uint64).copy()
    v = np.ascontiguousarray(values, dtype=np.uint32).copy()
    lib().gso_sort_pairs(_p(k), _p(v), k.size, threads)
    return k, v


def density_accumulate(grads: np.ndarray, accum: np.ndarray, count: np.ndarray,
                       pos_accum: np.ndarray) -> None:
    g = np.ascontiguousarray(grads, dtype=np.float32)
    lib().gso_density_accumulate(_p(g), g.shape[0], _p(accum), _p(count), _p(pos_accum))


def density_apply(gaussians: np.ndarray, accum: np.ndarray, count: np.ndarray, iteration: int,
                  scene_extent: float, focal: float, image_width: float, avg_depth: float,
                  seed: int, max_gaussians: int = 0):
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    n = g.shape[0]
    out = np.zeros((max(2 * n, 1), 28), dtype=np.float32)
    markers = np.zeros(max(n, 1), dtype=np.uint32)
    stats = np.zeros(4, dtype=np.uint32)
    m = lib().gso_density_apply(_p(g), n, _p(np.ascontiguousarray(accum, np.float32)),
                                _p(np.ascontiguousarray(count, np.uint32)), iteration,
                                scene_extent, focal, image_width, avg_depth, seed, max_gaussians,
                                _p(out), _p(markers), _p(stats))
    return out[:m], markers[:n], dict(num_pruned=int(stats[0]), num_cloned=int(stats[1]),
                                       num_split=int(stats[2]))


class AdamState:
    """The reference optimizer's state in its own layout (optimizer.mm:46-73)."""

    def __init__(self, n: int):
        self.n = n
        self.t = 0
        z = lambda k: np.zeros(max(n * k, 1), dtype=np.float32)  # noqa: E731
        self.m_pos, self.m_scale, self.m_rot, self.m_op, self.m_sh = z(3), z(3), z(4), z(1), z(12)
        self.v_pos, self.v_scale, self.v_rot, self.v_op, self.v_sh = z(3), z(3), z(4), z(1), z(12)

    def records(self, which: str) -> np.ndarray:
        """(n, 24) in the library's moment-record layout: pos xyz, opacity, scale xyz, 0,
        rotation, sh 0..11."""
        pre = "m_" if which == "m" else "v_"
        g = lambda k: getattr(self, pre + k)  # noqa: E731
        r = np.zeros((self.n, 24), dtype=np.float32)
        r[:, 0:3] = g("pos")[:3 * self.n].reshape(-1, 3)
        r[:, 3] = g("op")[:self.n]
        r[:, 4:7] = g("scale")[:3 * self.n].reshape(-1, 3)
        r[:, 8:12] = g("rot")[:4 * self.n].reshape(-1, 4)
        r[:, 12:24] = g("sh")[:12 * self.n].reshape(-1, 12)
        return r

    def set_records(self, m: np.ndarray, v: np.ndarray) -> None:
        """Replace the state (n may change) from (n, 24) records in the layout of records()."""
        n = m.shape[0]
        self.n = n
        for pre, r in (("m_", m), ("v_", v)):
            r = np.asarray(r, dtype=np.float32)
            setattr(self, pre + "pos", np.ascontiguousarray(r[:, 0:3]).reshape(-1).copy() if n else np.zeros(1, np.float32))
            setattr(self, pre + "op", np.ascontiguousarray(r[:, 3]).copy() if n else np.zeros(1, np.float32))
            setattr(self, pre + "scale", np.ascontiguousarray(r[:, 4:7]).reshape(-1).copy() if n else np.zeros(1, np.float32))
            setattr(self, pre + "rot", np.ascontiguousarray(r[:, 8:12]).reshape(-1).copy() if n else np.zeros(1, np.float32))
            setattr(self, pre + "sh", np.ascontiguousarray(r[:, 12:24]).reshape(-1).copy() if n else np.zeros(1, np.float32))


def bias_corrections(t: int, beta1: float = 0.9, beta2: float = 0.999):
    """1 - beta^t (shaders.metal:579-580) with a correctly rounded pow, then a float subtraction."""
    b1, b2 = float(np.float32(beta1)), float(np.float32(beta2))
    p1, p2 = np.float32(b1 ** t), np.float32(b2 ** t)
    return float(np.float32(1.0) - p1), float(np.float32(1.0) - p2)


def adam_step(gaussians: np.ndarray, grads: np.ndarray, state: AdamState, lrs,
              beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8) -> None:
    """AdamOptimizer::step (optimizer.mm:241-296) in place on `gaussians` and `state`."""
    assert gaussians.dtype == np.float32 and gaussians.flags.c_contiguous
    n = gaussians.shape[0]
    gr = np.ascontiguousarray(grads, dtype=np.float32)
    state.t += 1
    bc1, bc2 = bias_corrections(state.t, beta1, beta2)
    lr = np.ascontiguousarray(lrs, dtype=np.float32)
    lib().gso_adam_step(_p(gaussians), _p(gr), n, _p(state.m_pos), _p(state.m_scale),
                        _p(state.m_rot), _p(state.m_op), _p(state.m_sh), _p(state.v_pos),
                        _p(state.v_scale), _p(state.v_rot), _p(state.v_op), _p(state.v_sh),
                        _p(lr), beta1, beta2, eps, bc1, bc2)


def opacity_reset(gaussians: np.ndarray, max_raw: float = -4.6) -> None:
    lib().gso_opacity_reset(_p(gaussians), gaussians.shape[0], max_raw)


def loss(rendered: np.ndarray, gt: np.ndarray, lambda_dssim: float = 0.2, threads: int = 8):
    """MTLEngine::computeLoss kernels (shaders.metal:320-510): (mean combined loss, maps[3,h,w])."""
    r = np.ascontiguousarray(rendered, dtype=np.uint32)
    g = np.ascontiguousarray(gt, dtype=np.uint32)
    h, w = r.shape
    maps = np.zeros((3, h, w), dtype=np.float32)
    m = lib().gso_loss(_p(r), _p(g), w, h, lambda_dssim, _p(maps), threads)
    return float(m), maps


def expf(x: float) -> float:
    return float(lib().gso_expf(x))


def half(x: float) -> float:
    return float(lib().gso_half(x))
