"""Host-side mirror of the reference's operator interface for the hot path.

  TiledRasterizer    <- GuassianSplatting/tiled_rasterizer.hpp:56-124
                        (constructor(device, maxGaussians), forward, backward)
  DensityController  <- GuassianSplatting/density_control.hpp:22-48
                        (accumulateGradients, apply, resetAccumulator, setSceneExtent)

Buffers are torch tensors on a HIP device (torch is plumbing here: device memory and streams);
the compute is the HIP library behind the C-ABI (include/gs_rasterizer.h). Record tensors use the
reference layouts: Gaussians (N, 28) float32, gradients (N, 28) float32, RGBA8 images (H, W) int32
holding packed R | G<<8 | B<<16 | A<<24, uniforms a 60-float array (240 B).
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_size_t, c_uint64, c_void_p

import numpy as np

from . import _lib
from .scene import D_FLOATS, G_FLOATS, PROJECTED_DTYPE, ROW_FLOATS, U_FLOATS, tiles_for


def _torch():
    import torch
    return torch


def _stream_ptr(stream) -> int:
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _uniform_buffer(uniforms) -> ctypes.Array:
    u = np.ascontiguousarray(np.asarray(uniforms, dtype=np.float32).reshape(-1))
    if u.size != U_FLOATS:
        raise ValueError(f"uniforms must have {U_FLOATS} float32 entries (240 B), got {u.size}")
    return (ctypes.c_float * U_FLOATS).from_buffer_copy(u.tobytes())


def _check_records(t, name: str, floats: int):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TypeError(f"{name} must be a device tensor")
    if t.dtype != torch.float32 or t.dim() != 2 or t.shape[1] != floats or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous (N, {floats}) float32 tensor")


def _check_image(t, name: str, w: int, h: int):
    torch = _torch()
    if t.device.type != "cuda" or t.dtype != torch.int32 or tuple(t.shape) != (h, w) \
            or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous ({h}, {w}) int32 device tensor")


class TiledRasterizer:
    """MI355X tiled rasterizer (tiled_rasterizer.hpp:56-124).

    forward: project -> tile keys -> (tile|depth) radix sort -> tile ranges -> front-to-back
    blend. backward: reverse traversal + per-Gaussian chain into GaussianGradients. As in the
    reference, backward must directly follow forward with the same Gaussians and uniforms.
    """

    def __init__(self, max_gaussians: int = 0, device: int = 0, max_width: int = 0,
                 max_height: int = 0):
        self._h = c_void_p()
        self.device = device
        _lib.call("gs_create", device, max_gaussians, max_width, max_height, byref(self._h))
        self._w = self._hgt = 0
        self._n = 0

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().gs_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve_pairs(self, max_pairs: int) -> None:
        """Pre-size the pair buffers; at >= n*min(256, tiles) the frame is sync-free."""
        _lib.call("gs_reserve_pairs", self._h, max_pairs)

    def set_tile_sort_path(self, mode: int) -> None:
        """0 automatic, 1 one-pass counting sort (tiles <= 12288), 2 two-pass LSD (gs_set_tile_sort_path)."""
        _lib.call("gs_set_tile_sort_path", self._h, int(mode))

    def set_chain_compact(self, mode: int) -> None:
        """Chain kernel: < 0 automatic (compacting above 8 pairs per Gaussian), 0 plain, 1 compacting
        (gs_set_chain_compact)."""
        _lib.call("gs_set_chain_compact", self._h, int(mode))

    def set_depth_sort(self, mode: int) -> None:
        """gs_set_depth_sort: 0 automatic, 1 global depth sort, 2 per-tile depth sort."""
        _lib.call("gs_set_depth_sort", self._h, int(mode))

    def set_backward_split(self, tiles: int) -> None:
        """Tiles whose backward runs as two list halves: < 0 automatic (all), 0 off (gs_set_backward_split)."""
        _lib.call("gs_set_backward_split", self._h, int(tiles))

    def forward(self, gaussians, uniforms, output, rgb_out=None, stream=None) -> None:
        """tiled_rasterizer.hpp:63-67. `output` is the (H, W) int32 RGBA8 render target."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        h, w = int(output.shape[0]), int(output.shape[1])
        _check_image(output, "output", w, h)
        if rgb_out is not None:
            torch = _torch()
            if rgb_out.dtype != torch.float32 or tuple(rgb_out.shape) != (h, w, 3):
                raise ValueError("rgb_out must be a (H, W, 3) float32 device tensor")
        u = _uniform_buffer(uniforms)
        n = int(gaussians.shape[0])
        _lib.call("gs_forward", self._h, _stream_ptr(stream), gaussians.data_ptr(), n, u, w, h,
                  output.data_ptr(), rgb_out.data_ptr() if rgb_out is not None else None)
        self._w, self._hgt, self._n = w, h, n

    def backward(self, gaussians, gradients, uniforms, rendered, ground_truth,
                 stream=None) -> None:
        """tiled_rasterizer.hpp:69-75. Every gradient record [0, N) is written."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        _check_records(gradients, "gradients", D_FLOATS)
        if gradients.shape[0] < gaussians.shape[0]:
            raise ValueError("gradients has fewer records than gaussians")
        h, w = int(rendered.shape[0]), int(rendered.shape[1])
        _check_image(rendered, "rendered", w, h)
        _check_image(ground_truth, "ground_truth", w, h)
        u = _uniform_buffer(uniforms)
        _lib.call("gs_backward", self._h, _stream_ptr(stream), gaussians.data_ptr(),
                  gradients.data_ptr(), int(gaussians.shape[0]), u, rendered.data_ptr(),
                  ground_truth.data_ptr())

    def backward_rows(self, gaussians, rows, viewspace, uniforms, rendered, ground_truth,
                      stream=None) -> None:
        """gs_backward_packed: the gradients as (N, 14) rows (ROW_FLOATS; the data-parallel path
        reduces these) and, when `viewspace` is an (N, 2) tensor, the per-view screen-space gradient."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        _check_records(rows, "rows", ROW_FLOATS)
        n = int(gaussians.shape[0])
        if rows.shape[0] < n or (viewspace is not None and (viewspace.shape[0] < n)):
            raise ValueError("rows / viewspace have fewer entries than gaussians")
        if viewspace is not None:
            _check_records(viewspace, "viewspace", 2)
        h, w = int(rendered.shape[0]), int(rendered.shape[1])
        _check_image(rendered, "rendered", w, h)
        _check_image(ground_truth, "ground_truth", w, h)
        _lib.call("gs_backward_packed", self._h, _stream_ptr(stream), gaussians.data_ptr(), rows.data_ptr(),
                  viewspace.data_ptr() if viewspace is not None else None, n, _uniform_buffer(uniforms),
                  rendered.data_ptr(), ground_truth.data_ptr())

    def backward_step(self, gaussians, uniforms, rendered, ground_truth, adam: "AdamOptimizer",
                      density: "DensityController | None" = None, lrs=None, stream=None) -> None:
        """gs_backward_step: the backward of one training step fused through the optimizer --
        per Gaussian the chain, the density statistics (when `density` is given) and Adam in place
        on `gaussians` (t += 1). Equal bit for bit to backward_rows + density.accumulate_rows +
        adam.step_rows; no gradient rows are written."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        h, w = int(rendered.shape[0]), int(rendered.shape[1])
        _check_image(rendered, "rendered", w, h)
        _check_image(ground_truth, "ground_truth", w, h)
        lr = (ctypes.c_float * 5)(*[float(x) for x in (AdamOptimizer.DEFAULT_LRS if lrs is None else lrs)])
        _lib.call("gs_backward_step", self._h, _stream_ptr(stream), gaussians.data_ptr(), int(gaussians.shape[0]),
                  _uniform_buffer(uniforms), rendered.data_ptr(), ground_truth.data_ptr(),
                  density._h if density is not None else None, adam._h, lr)

    def frame_stats(self) -> dict:
        s = _lib.GsFrameStats()
        _lib.call("gs_frame_stats", self._h, byref(s))
        return {k: getattr(s, k) for k, _ in s._fields_ if not k.startswith("_")}

    # ---- debug getters (parity tests) ------------------------------------------------
    def num_pairs(self) -> int:
        v = c_uint64()
        _lib.call("gs_debug_num_pairs", self._h, byref(v))
        return int(v.value)

    def sorted_pairs(self, stream=None):
        torch = _torch()
        p = self.num_pairs()
        keys = torch.empty(max(p, 1), dtype=torch.int64, device=f"cuda:{self.device}")
        vals = torch.empty(max(p, 1), dtype=torch.int32, device=f"cuda:{self.device}")
        _lib.call("gs_debug_sorted_pairs", self._h, _stream_ptr(stream), keys.data_ptr(),
                  vals.data_ptr(), p)
        torch.cuda.synchronize()
        return (keys[:p].cpu().numpy().view(np.uint64), vals[:p].cpu().numpy().view(np.uint32))

    def tile_ranges(self, stream=None) -> np.ndarray:
        torch = _torch()
        tx, ty = tiles_for(self._w, self._hgt)
        out = torch.empty((tx * ty, 2), dtype=torch.int32, device=f"cuda:{self.device}")
        _lib.call("gs_debug_tile_ranges", self._h, _stream_ptr(stream), out.data_ptr(), tx * ty)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)

    def last_idx(self, stream=None) -> np.ndarray:
        torch = _torch()
        out = torch.empty((self._hgt, self._w), dtype=torch.int32, device=f"cuda:{self.device}")
        _lib.call("gs_debug_last_idx", self._h, _stream_ptr(stream), out.data_ptr(),
                  self._w * self._hgt)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)

    def projected(self, stream=None) -> np.ndarray:
        torch = _torch()
        out = torch.empty((max(self._n, 1), 22), dtype=torch.float32, device=f"cuda:{self.device}")
        _lib.call("gs_debug_projected", self._h, _stream_ptr(stream), out.data_ptr(), self._n)
        torch.cuda.synchronize()
        return out[: self._n].cpu().numpy().view(PROJECTED_DTYPE).reshape(-1)


class DensityController:
    """density_control.hpp:22-48 on the GPU.

    `capacity` only pre-sizes the accumulators (they grow with the largest count seen).
    `max_gaussians` is the population cap of apply — the reference's MAX_GAUSSIANS (1.5M,
    density_control.mm:27, 360-382), whose excess clones then splits are dropped in index order;
    0 (the default) means unlimited."""

    def __init__(self, capacity: int = 0, device: int = 0, max_gaussians: int = 0):
        self._h = c_void_p()
        self.device = device
        _lib.call("gs_density_create", device, capacity, byref(self._h))
        if max_gaussians:
            self.set_max_gaussians(max_gaussians)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().gs_density_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene_extent(self, extent: float) -> None:
        _lib.call("gs_density_set_scene_extent", self._h, float(extent))

    def set_max_gaussians(self, max_gaussians: int) -> None:
        _lib.call("gs_density_set_max_gaussians", self._h, int(max_gaussians))

    def reset_accumulator(self, n: int, stream=None) -> None:
        _lib.call("gs_density_reset", self._h, _stream_ptr(stream), int(n))

    def accumulate_gradients(self, gradients, n: int | None = None, stream=None) -> None:
        _check_records(gradients, "gradients", D_FLOATS)
        n = int(gradients.shape[0]) if n is None else int(n)
        _lib.call("gs_density_accumulate", self._h, _stream_ptr(stream), gradients.data_ptr(), n)

    def accumulate_rows(self, rows, viewspace, n: int | None = None, stream=None) -> None:
        """gs_density_accumulate_rows: the same statistics from gradient rows + viewspace rows."""
        _check_records(rows, "rows", ROW_FLOATS)
        _check_records(viewspace, "viewspace", 2)
        n = int(rows.shape[0]) if n is None else int(n)
        _lib.call("gs_density_accumulate_rows", self._h, _stream_ptr(stream), rows.data_ptr(),
                  viewspace.data_ptr(), n)

    def accumulate_rows_range(self, rows, viewspace, first: int, count: int, stream=None) -> None:
        """gs_density_accumulate_rows_range: accumulate_rows for the Gaussians [first, first + count)
        (rows / viewspace are the whole (N, 14) / (N, 2) buffers)."""
        _check_records(rows, "rows", ROW_FLOATS)
        _check_records(viewspace, "viewspace", 2)
        first, count = int(first), int(count)
        if first < 0 or count < 0 or first + count > min(rows.shape[0], viewspace.shape[0]):
            raise ValueError("accumulate_rows_range: range outside the buffers")
        _lib.call("gs_density_accumulate_rows_range", self._h, _stream_ptr(stream), rows.data_ptr(),
                  viewspace.data_ptr(), first, count)

    def read(self, n: int, stream=None):
        torch = _torch()
        dev = f"cuda:{self.device}"
        acc = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        cnt = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        pos = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
        _lib.call("gs_density_read", self._h, _stream_ptr(stream), acc.data_ptr(), cnt.data_ptr(),
                  pos.data_ptr(), n)
        torch.cuda.synchronize()
        return (acc[:n].cpu().numpy(), cnt[:n].cpu().numpy().view(np.uint32),
                pos[:n].cpu().numpy())

    def statistics(self, n: int, stream=None):
        """The accumulators as device tensors (accum f32[n], count i32[n], pos_accum f32[n, 3])."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        acc = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        cnt = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        pos = torch.empty((max(n, 1), 3), dtype=torch.float32, device=dev)
        _lib.call("gs_density_read", self._h, _stream_ptr(stream), acc.data_ptr(), cnt.data_ptr(),
                  pos.data_ptr(), n)
        return acc[:n], cnt[:n], pos[:n]

    def set_statistics(self, accum, count, pos_accum, n: int, stream=None) -> None:
        """Overwrite the accumulators (e.g. with their all-reduced sum over ranks)."""
        _lib.call("gs_density_write", self._h, _stream_ptr(stream), accum.data_ptr(),
                  count.data_ptr(), pos_accum.data_ptr(), n)

    def apply(self, gaussians, iteration: int, focal_length: float = 500.0,
              image_width: float = 800.0, avg_depth: float = 5.0, seed: int = 0, stream=None):
        """density_control.hpp:26-37. Returns (new Gaussians tensor, DensityStats dict)."""
        torch = _torch()
        _check_records(gaussians, "gaussians", G_FLOATS)
        out_ptr = c_void_p()
        out_n = c_size_t()
        st = _lib.GsDensityStats()
        _lib.call("gs_density_apply", self._h, _stream_ptr(stream), gaussians.data_ptr(),
                  int(gaussians.shape[0]), byref(out_ptr), byref(out_n), int(iteration),
                  float(focal_length), float(image_width), float(avg_depth), int(seed), byref(st))
        n = int(out_n.value)
        new = torch.empty((max(n, 1), G_FLOATS), dtype=torch.float32,
                          device=gaussians.device)
        if n:
            torch.cuda.synchronize()
            _copy_device(new.data_ptr(), out_ptr.value, n * G_FLOATS * 4)
        _lib.call("gs_free", out_ptr)
        return new[:n], {"num_pruned": st.num_pruned, "num_cloned": st.num_cloned,
                         "num_split": st.num_split}


class AdamOptimizer:
    """optimizer.hpp:22-95 on the GPU: Adam over the Gaussian records in place.

    lrs default to the reference's AdamOptimizer::step defaults (optimizer.hpp:29-41)."""

    DEFAULT_LRS = (0.00016, 0.005, 0.001, 0.05, 0.0025)

    def __init__(self, max_gaussians: int = 0, device: int = 0):
        self._h = c_void_p()
        self.device = device
        _lib.call("gs_adam_create", device, max_gaussians, byref(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().gs_adam_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def step(self, gaussians, gradients, lrs=DEFAULT_LRS, n: int | None = None, stream=None) -> None:
        _check_records(gaussians, "gaussians", G_FLOATS)
        _check_records(gradients, "gradients", D_FLOATS)
        n = int(gaussians.shape[0]) if n is None else int(n)
        lr = (ctypes.c_float * 5)(*[float(x) for x in lrs])
        _lib.call("gs_adam_step", self._h, _stream_ptr(stream), gaussians.data_ptr(),
                  gradients.data_ptr(), n, lr)

    def step_rows(self, gaussians, rows, lrs=DEFAULT_LRS, first: int = 0, count: int | None = None,
                  stream=None) -> None:
        """gs_adam_step_rows: rows[k] is the gradient of Gaussian first + k (k < count). One call is
        one optimizer step (t += 1): a step split over several ranges takes begin_step +
        step_rows_range instead."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        _check_records(rows, "rows", ROW_FLOATS)
        count = int(rows.shape[0]) if count is None else int(count)
        if first + count > gaussians.shape[0] or count > rows.shape[0]:
            raise ValueError("step_rows: range outside the buffers")
        lr = (ctypes.c_float * 5)(*[float(x) for x in lrs])
        _lib.call("gs_adam_step_rows", self._h, _stream_ptr(stream), gaussians.data_ptr(), rows.data_ptr(),
                  int(first), count, lr)

    def begin_step(self) -> None:
        """gs_adam_begin_step: t += 1 for an optimizer step applied in several ranges."""
        _lib.call("gs_adam_begin_step", self._h)

    def step_rows_range(self, gaussians, rows, lrs=DEFAULT_LRS, first: int = 0, count: int | None = None,
                        stream=None) -> None:
        """gs_adam_step_rows_range: step_rows for [first, first + count) at the timestep of the last
        begin_step, without advancing it (one step split over chunks)."""
        _check_records(gaussians, "gaussians", G_FLOATS)
        _check_records(rows, "rows", ROW_FLOATS)
        count = int(rows.shape[0]) if count is None else int(count)
        if first + count > gaussians.shape[0] or count > rows.shape[0]:
            raise ValueError("step_rows_range: range outside the buffers")
        lr = (ctypes.c_float * 5)(*[float(x) for x in lrs])
        _lib.call("gs_adam_step_rows_range", self._h, _stream_ptr(stream), gaussians.data_ptr(),
                  rows.data_ptr(), int(first), count, lr)

    @property
    def timestep(self) -> int:
        t = ctypes.c_uint32()
        _lib.call("gs_adam_timestep", self._h, byref(t))
        return int(t.value)

    def reset(self, stream=None) -> None:
        _lib.call("gs_adam_reset", self._h, _stream_ptr(stream))

    def resize_if_needed(self, n: int, stream=None) -> None:
        _lib.call("gs_adam_resize", self._h, _stream_ptr(stream), int(n))

    def reset_state_for_new_gaussians(self, start: int, n: int, stream=None) -> None:
        _lib.call("gs_adam_reset_new", self._h, _stream_ptr(stream), int(start), int(n))

    def reset_opacity_momentum(self, n: int, stream=None) -> None:
        _lib.call("gs_adam_reset_opacity_momentum", self._h, _stream_ptr(stream), int(n))

    def reset_scale_momentum(self, n: int, stream=None) -> None:
        _lib.call("gs_adam_reset_scale_momentum", self._h, _stream_ptr(stream), int(n))

    def follow_density(self, density: "DensityController", n_in: int, n_out: int, stream=None) -> None:
        _lib.call("gs_adam_follow_density", self._h, _stream_ptr(stream), density._h, int(n_in),
                  int(n_out))

    def state(self, n: int, stream=None):
        """(m, v) as (n, 24) float32 arrays: pos xyz, opacity, log-scale xyz, 0, rotation, sh."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        m = torch.empty((max(n, 1), 24), dtype=torch.float32, device=dev)
        v = torch.empty((max(n, 1), 24), dtype=torch.float32, device=dev)
        _lib.call("gs_adam_read_state", self._h, _stream_ptr(stream), m.data_ptr(), v.data_ptr(), int(n))
        torch.cuda.synchronize()
        return m[:n].cpu().numpy(), v[:n].cpu().numpy()


    def state_tensors(self, n: int, stream=None):
        """(m, v) as (n, 24) float32 device tensors (no host copy)."""
        torch = _torch()
        dev = f"cuda:{self.device}"
        m = torch.empty((max(n, 1), 24), dtype=torch.float32, device=dev)
        v = torch.empty((max(n, 1), 24), dtype=torch.float32, device=dev)
        _lib.call("gs_adam_read_state", self._h, _stream_ptr(stream), m.data_ptr(), v.data_ptr(), int(n))
        return m[:n], v[:n]

    def set_state(self, m, v, n: int, stream=None) -> None:
        """Overwrite the moments of [0, n) with (n, 24) float32 device tensors."""
        n = int(n)
        for t, name in ((m, "m"), (v, "v")):
            _check_records(t, name, 24)
            if t.shape[0] < n:
                raise ValueError(f"set_state: {name} holds {t.shape[0]} rows, fewer than n = {n}")
            if t.device.index != self.device:
                raise ValueError(f"set_state: {name} is on cuda:{t.device.index}, the optimizer on cuda:{self.device}")
        _lib.call("gs_adam_write_state", self._h, _stream_ptr(stream), m.data_ptr(), v.data_ptr(), int(n))


class Loss:
    """MTLEngine::computeLoss (mtl_engine.mm:769-853): (1 - lambda) L1 + lambda D-SSIM, mean."""

    def __init__(self, device: int = 0):
        self._h = c_void_p()
        self.device = device
        _lib.call("gs_loss_create", device, byref(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().gs_loss_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compute(self, rendered, gt, lambda_dssim: float = 0.2, maps=None, out=None, stream=None):
        """Returns a 1-element float32 device tensor with the mean combined loss (stream-ordered);
        `maps`, if given, is a (3, H, W) float32 device tensor for the L1 / D-SSIM / combined maps."""
        torch = _torch()
        h, w = int(rendered.shape[0]), int(rendered.shape[1])
        _check_image(rendered, "rendered", w, h)
        _check_image(gt, "gt", w, h)
        if out is None:
            out = torch.empty(1, dtype=torch.float32, device=rendered.device)
        mp = 0
        if maps is not None:
            if maps.dtype != torch.float32 or tuple(maps.shape) != (3, h, w) or not maps.is_contiguous():
                raise ValueError("maps must be a contiguous (3, H, W) float32 tensor")
            mp = maps.data_ptr()
        _lib.call("gs_loss_compute", self._h, _stream_ptr(stream), rendered.data_ptr(), gt.data_ptr(),
                  w, h, float(lambda_dssim), out.data_ptr(), mp or None)
        return out


def unpack_gradients(rows, viewspace, gradients, n: int | None = None, stream=None) -> None:
    """gs_unpack_gradients: (N, 14) rows + (N, 2) viewspace (None = zero) -> (N, 28) records."""
    _check_records(rows, "rows", ROW_FLOATS)
    _check_records(gradients, "gradients", D_FLOATS)
    if viewspace is not None:
        _check_records(viewspace, "viewspace", 2)
    n = int(rows.shape[0]) if n is None else int(n)
    _lib.call("gs_unpack_gradients", _stream_ptr(stream), rows.data_ptr(),
              viewspace.data_ptr() if viewspace is not None else None, gradients.data_ptr(), n)


def opacity_reset(gaussians, max_raw: float = -4.6, n: int | None = None, stream=None) -> None:
    """mtl_engine.mm:1173-1186: raw opacity = min(raw opacity, max_raw)."""
    _check_records(gaussians, "gaussians", G_FLOATS)
    n = int(gaussians.shape[0]) if n is None else int(n)
    _lib.call("gs_opacity_reset", _stream_ptr(stream), gaussians.data_ptr(), n, float(max_raw))


def _copy_device(dst: int, src: int, nbytes: int) -> None:
    """Device-to-device copy through the HIP runtime (the library's buffer is not a tensor)."""
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [c_void_p, c_void_p, c_size_t, ctypes.c_int]
    rc = hip.hipMemcpy(c_void_p(dst), c_void_p(src), c_size_t(nbytes), 3)  # DeviceToDevice
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed with {rc}")
