"""ctypes binding of the C-ABI in include/gs_rasterizer.h.

The shared library is built in-tree (``make`` -> gaussiansplatting_amd/lib/libgs_mi355x.so) so
that it travels with the repository snapshot. There is no fallback: if the library is missing
every entry point raises, so a GPU run can never silently take a non-HIP path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# GS_MI355X_LIB selects another in-tree build of the same library (kernel A/B experiments).
LIB_PATH = os.path.join(_HERE, "lib", os.environ.get("GS_MI355X_LIB", "libgs_mi355x.so"))

GS_OK = 0
GS_E_INVALID = -1
GS_E_HIP = -2
GS_E_NOMEM = -3
GS_E_STATE = -4
GS_E_CAPACITY = -5


class GsFrameStats(ctypes.Structure):
    _fields_ = [
        ("num_pairs", c_uint64),
        ("pair_capacity", c_uint64),
        ("num_visible", c_uint32),
        ("num_tiles", c_uint32),
        ("width", c_uint32),
        ("height", c_uint32),
        ("sort_passes_depth", c_uint32),
        ("sort_passes_tile", c_uint32),
        ("overflowed", c_uint32),
        ("scan_errors", c_uint32),
        ("tile_sort_path", c_uint32),
        ("_pad", c_uint32),
        ("fwd_walked_entries", c_uint64),
        ("bwd_walked_entries", c_uint64),
        ("reached_gaussians", c_uint64),
        ("reached_slots", c_uint64),
    ]


class GsDensityStats(ctypes.Structure):
    _fields_ = [
        ("num_pruned", c_uint32),
        ("num_cloned", c_uint32),
        ("num_split", c_uint32),
        ("_pad", c_uint32),
    ]


class GsColmapCamera(ctypes.Structure):
    _fields_ = [("id", c_uint32), ("width", c_uint32), ("height", c_uint32), ("model", ctypes.c_int32),
                ("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float)]


class GsColmapImage(ctypes.Structure):
    _fields_ = [("id", c_uint32), ("camera_id", c_uint32), ("rotation", c_float * 4),
                ("translation", c_float * 3), ("_pad", c_float), ("name", ctypes.c_char * 256)]


class GsColmapPoint(ctypes.Structure):
    _fields_ = [("position", c_float * 3), ("color", c_float * 3), ("error", c_float)]


# name -> (restype, argtypes); exactly the functions include/gs_rasterizer.h declares
SIGNATURES = {
    "gs_last_error": (c_char_p, []),
    "gs_abi_version": (c_int, []),
    "gs_create": (c_int, [c_int, c_uint32, c_uint32, c_uint32, POINTER(c_void_p)]),
    "gs_destroy": (c_int, [c_void_p]),
    "gs_reserve_pairs": (c_int, [c_void_p, c_uint64]),
    "gs_set_tile_sort_path": (c_int, [c_void_p, c_int]),
    "gs_set_backward_split": (c_int, [c_void_p, c_int]),
    "gs_set_chain_compact": (c_int, [c_void_p, c_int]),
    "gs_set_depth_sort": (c_int, [c_void_p, c_int]),
    "gs_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_uint32, c_uint32,
                           c_void_p, c_void_p]),
    "gs_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                            c_void_p, c_void_p]),
    "gs_backward_packed": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p,
                                   c_void_p, c_void_p]),
    "gs_unpack_gradients": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_backward_blend": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                  c_void_p]),
    "gs_backward_chain": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                  c_void_p, c_size_t, c_size_t]),
    "gs_backward_step": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p]),
    "gs_set_stage_timing": (c_int, [c_void_p, c_int]),
    "gs_stage_times": (c_int, [c_void_p, POINTER(ctypes.c_double), POINTER(c_uint32), c_int]),
    "gs_frame_stats": (c_int, [c_void_p, POINTER(GsFrameStats)]),
    "gs_debug_num_pairs": (c_int, [c_void_p, POINTER(c_uint64)]),
    "gs_debug_sorted_pairs": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]),
    "gs_debug_tile_ranges": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32]),
    "gs_debug_last_idx": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64]),
    "gs_debug_projected": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_debug_half_exp_check": (c_int, [c_int, POINTER(c_uint32), POINTER(c_uint32)]),
    "gs_debug_float_exp_check": (c_int, [c_int, POINTER(c_float)]),
    "gs_debug_copy_bandwidth": (c_int, [c_int, c_uint64, c_int, POINTER(ctypes.c_double), POINTER(ctypes.c_double),
                                        c_int]),
    "gs_density_create": (c_int, [c_int, c_uint32, POINTER(c_void_p)]),
    "gs_density_destroy": (c_int, [c_void_p]),
    "gs_density_set_max_gaussians": (c_int, [c_void_p, c_uint64]),
    "gs_density_set_scene_extent": (c_int, [c_void_p, c_float]),
    "gs_density_reset": (c_int, [c_void_p, c_void_p, c_size_t]),
    "gs_density_accumulate": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_density_accumulate_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_density_accumulate_rows_range": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                                 c_size_t]),
    "gs_density_read": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_density_write": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_density_apply": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, POINTER(c_void_p),
                                 POINTER(c_size_t), c_uint64, c_float, c_float, c_float,
                                 c_uint64, POINTER(GsDensityStats)]),
    "gs_adam_create": (c_int, [c_int, c_uint32, POINTER(c_void_p)]),
    "gs_adam_destroy": (c_int, [c_void_p]),
    "gs_adam_reset": (c_int, [c_void_p, c_void_p]),
    "gs_adam_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, POINTER(c_float)]),
    "gs_adam_step_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_size_t,
                                  POINTER(c_float)]),
    "gs_adam_begin_step": (c_int, [c_void_p]),
    "gs_adam_step_rows_range": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_size_t,
                                        POINTER(c_float)]),
    "gs_adam_timestep": (c_int, [c_void_p, POINTER(c_uint32)]),
    "gs_adam_resize": (c_int, [c_void_p, c_void_p, c_size_t]),
    "gs_adam_reset_new": (c_int, [c_void_p, c_void_p, c_size_t, c_size_t]),
    "gs_adam_reset_opacity_momentum": (c_int, [c_void_p, c_void_p, c_size_t]),
    "gs_adam_reset_scale_momentum": (c_int, [c_void_p, c_void_p, c_size_t]),
    "gs_adam_follow_density": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t]),
    "gs_adam_read_state": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_adam_write_state": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    "gs_opacity_reset": (c_int, [c_void_p, c_void_p, c_size_t, c_float]),
    "gs_loss_create": (c_int, [c_int, POINTER(c_void_p)]),
    "gs_loss_destroy": (c_int, [c_void_p]),
    "gs_loss_compute": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint32, c_float,
                                c_void_p, c_void_p]),
    "gs_colmap_load": (c_int, [c_char_p, POINTER(c_void_p)]),
    "gs_colmap_free": (c_int, [c_void_p]),
    "gs_colmap_counts": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint64)]),
    "gs_colmap_camera": (c_int, [c_void_p, c_uint32, POINTER(GsColmapCamera)]),
    "gs_colmap_camera_by_id": (c_int, [c_void_p, c_uint32, POINTER(GsColmapCamera)]),
    "gs_colmap_image": (c_int, [c_void_p, c_uint32, POINTER(GsColmapImage)]),
    "gs_colmap_points": (c_int, [c_void_p, c_void_p, c_uint64]),
    "gs_colmap_camera_position": (c_int, [POINTER(GsColmapImage), POINTER(c_float)]),
    "gs_colmap_scene_extent": (c_int, [c_void_p, POINTER(c_float)]),
    "gs_gaussians_from_colmap": (c_int, [c_void_p, c_float, c_void_p, c_uint64, POINTER(c_uint64)]),
    "gs_colmap_uniforms": (c_int, [POINTER(GsColmapCamera), POINTER(GsColmapImage), c_uint32, c_uint32,
                                   c_void_p]),
    "gs_ply_load": (c_int, [c_char_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "gs_ply_save": (c_int, [c_char_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "gs_ppm_save": (c_int, [c_char_p, c_void_p, c_uint32, c_uint32]),
    "gs_ppm_load": (c_int, [c_char_p, c_void_p, c_uint64, POINTER(c_uint32), POINTER(c_uint32)]),
    "gs_free": (c_int, [c_void_p]),
}

_lib = None


class GsError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()' or `make`)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if name.startswith("gs_debug_") and not hasattr(handle, name):
                continue  # (an older A/B build without a newer diagnostics entry point)
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(code: int, where: str) -> None:
    if code != GS_OK:
        msg = lib().gs_last_error()
        raise GsError(code, where, msg.decode() if msg else "")


STAGES = ["project", "depth_sort", "offset_scan", "pair_emit", "tile_sort", "tile_ranges",
          "forward_blend", "backward_blend", "chain"]


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)
