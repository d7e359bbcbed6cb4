"""gaussiansplatting_amd — MI355X-native tiled 3D Gaussian Splatting rasterizer.

A drop-in for the hot path of ctaylo41/GaussianSplatting (TiledRasterizer forward/backward and
the DensityController hooks) built as hand-written gfx950 HIP kernels behind a C-ABI
(include/gs_rasterizer.h). See DESIGN.md.
"""
from .scene import (CONFIGS, GRAD_FIELDS, make_uniforms, rig_uniforms, synthetic_ground_truth,
                    synthetic_gaussians, tiles_for)

__all__ = [
    "CONFIGS", "GRAD_FIELDS", "make_uniforms", "rig_uniforms", "synthetic_ground_truth",
    "synthetic_gaussians", "tiles_for", "TiledRasterizer", "DensityController",
]


def __getattr__(name):
    # the HIP-backed classes load the shared library lazily (so CPU-only imports work)
    if name in ("TiledRasterizer", "DensityController"):
        from . import rasterizer
        return getattr(rasterizer, name)
    raise AttributeError(name)
