"""Record layouts, camera uniforms and the seeded synthetic scene.

Layouts are the reference's (include/gs_rasterizer.h):
  Gaussian          28 x f32 (112 B)  ply_loader.hpp:14-20
  GaussianGradients 28 x f32 (112 B)  gradients.hpp:11-31
  ProjectedGaussian 22 x 4 B (88 B)   tiled_rasterizer.hpp:24-39
  TiledUniforms     60 x 4 B (240 B)  tiled_rasterizer.hpp:42-53

Uniform construction mirrors MTLEngine::viewMatrixFromColmap / projectionFromColmap and the
uniform block of trainStep (mtl_engine.mm:637-682, 912-924).
"""
from __future__ import annotations

import math

import numpy as np

SH_C0 = 0.28209479177387814
TILE = 16

# float offsets inside the 28-float Gaussian record
G_POS, G_SCALE, G_ROT, G_OPACITY, G_SH = 0, 4, 8, 12, 13
G_FLOATS = 28
# float offsets inside the 28-float gradient record
D_POS, D_OPACITY, D_SCALE, D_ROT, D_SH, D_VIEWSPACE = 0, 3, 4, 8, 12, 24
D_FLOATS = 28
# the 16 fields the backward writes: (name, float offset)
GRAD_FIELDS = [
    ("position_x", 0), ("position_y", 1), ("position_z", 2), ("opacity", 3),
    ("scale_x", 4), ("scale_y", 5), ("scale_z", 6),
    ("rot_w", 8), ("rot_x", 9), ("rot_y", 10), ("rot_z", 11),
    ("sh0", 12), ("sh4", 16), ("sh8", 20), ("viewspace_x", 24), ("viewspace_y", 25),
]
P_FLOATS = 22
U_FLOATS = 60
# gradient rows (include/gs_rasterizer.h GS_GRAD_ROW_FLOATS): the GaussianGradients float offsets of
# row entries 0..13 -- what the data-parallel path reduces; viewspace (24, 25) travels per rank
ROW_FLOATS = 14
ROW_FIELDS = [0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 12, 16, 20]
VIEWSPACE_FIELDS = [24, 25]

PROJECTED_DTYPE = np.dtype([
    ("screen_pos", "<f4", (2,)), ("conic", "<f4", (3,)), ("depth", "<f4"), ("opacity", "<f4"),
    ("color", "<f4", (3,)), ("radius", "<f4"), ("tile_min_x", "<u4"), ("tile_min_y", "<u4"),
    ("tile_max_x", "<u4"), ("tile_max_y", "<u4"), ("_pad1", "<f4"), ("view_pos_xy", "<f4", (2,)),
    ("cov2d", "<f4", (3,)), ("_pad2", "<f4"),
])
assert PROJECTED_DTYPE.itemsize == 88


def tiles_for(w: int, h: int) -> tuple[int, int]:
    return (w + TILE - 1) // TILE, (h + TILE - 1) // TILE


# ---- SplitMix64 --------------------------------------------------------------------------
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, start: int, count: int) -> np.ndarray:
    """Outputs start..start+count-1 of the SplitMix64 stream seeded with `seed`."""
    with np.errstate(over="ignore"):
        k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniforms01(seed: int, start: int, count: int) -> np.ndarray:
    """u = (x >> 40) * 2^-24 in [0, 1), as float64 (exactly representable)."""
    return (splitmix64(seed, start, count) >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


DRAWS_PER_GAUSSIAN = 13


def synthetic_gaussians(n: int, seed: int, width: int, height: int,
                        focal: float | None = None) -> np.ndarray:
    """The seeded synthetic scene of SURVEY.md §8d, as an (n, 28) float32 Gaussian array.

    Per Gaussian (13 draws in this order): depth z = 2 + 8u; pixel (uW, uH) back-projected
    through fx = fy = W, cx = W/2, cy = H/2; three log-scales ln(sigma_px z / fx) with sigma_px
    log-uniform in [0.5, 5] px; a uniform unit quaternion (Shoemake) stored (w, x, y, z); raw
    opacity logit(U[0.05, 0.95]); SH DC (u - 0.5) / SH_C0, the other 9 SH values 0.
    """
    f = float(width) if focal is None else float(focal)
    return _synthetic(n, seed, width, height, f, f, width / 2.0, height / 2.0).astype(np.float32)


def synthetic_gaussians_camera(n: int, seed: int, width: int, height: int, fx: float, fy: float,
                               cx: float, cy: float, quat_wxyz=(1.0, 0.0, 0.0, 0.0),
                               translation=(0.0, 0.0, 0.0)) -> np.ndarray:
    """The same draws as synthetic_gaussians, back-projected through a general pinhole camera
    (fx != fy, any principal point) and placed in the world so that the COLMAP view
    [R | t] (view_matrix_from_colmap, mtl_engine.mm:637-659) sees them where the draws put them:
    p_world = R^T (p_cam - t). Most splats therefore land in that camera's image."""
    gc = _synthetic(n, seed, width, height, float(fx), float(fy), float(cx), float(cy))
    q = np.asarray(quat_wxyz, dtype=np.float64)
    view = view_matrix_from_colmap(q / np.linalg.norm(q), translation).astype(np.float64)
    rot = view[:3, :3].T  # [row][col]: p_cam = rot p_world + t
    t = np.asarray(translation, dtype=np.float64)
    gc[:, 0:3] = (gc[:, 0:3] - t) @ rot  # rows: (p - t)^T R = (R^T (p - t))^T
    return gc.astype(np.float32)


def _synthetic(n: int, seed: int, width: int, height: int, fx: float, fy: float, cx: float,
               cy: float) -> np.ndarray:
    """Camera-space draws of SURVEY.md §8d (float64, (n, 28))."""
    u = uniforms01(seed, 0, n * DRAWS_PER_GAUSSIAN).reshape(n, DRAWS_PER_GAUSSIAN)
    g = np.zeros((n, G_FLOATS), dtype=np.float64)
    f = fx
    z = 2.0 + 8.0 * u[:, 0]
    px = u[:, 1] * width
    py = u[:, 2] * height
    g[:, 0] = (px - cx) * z / fx
    g[:, 1] = (py - cy) * z / fy
    g[:, 2] = z
    for k in range(3):
        sigma = 0.5 * np.power(10.0, u[:, 3 + k])
        g[:, G_SCALE + k] = np.log(sigma * z / f)
    u1, u2, u3 = u[:, 6], u[:, 7], u[:, 8]
    a, b = np.sqrt(1.0 - u1), np.sqrt(u1)
    g[:, G_ROT + 0] = a * np.sin(2.0 * math.pi * u2)
    g[:, G_ROT + 1] = a * np.cos(2.0 * math.pi * u2)
    g[:, G_ROT + 2] = b * np.sin(2.0 * math.pi * u3)
    g[:, G_ROT + 3] = b * np.cos(2.0 * math.pi * u3)
    p = 0.05 + 0.9 * u[:, 9]
    g[:, G_OPACITY] = np.log(p / (1.0 - p))
    for k in range(3):
        g[:, G_SH + 4 * k] = (u[:, 10 + k] - 0.5) / SH_C0
    return g


def synthetic_ground_truth(seed: int, view: int, width: int, height: int) -> np.ndarray:
    """Uniform random RGBA8 (alpha 255) with stream seed + 1000 + view, packed R | G<<8 | B<<16."""
    x = splitmix64(seed + 1000 + view, 0, width * height * 3).reshape(height * width, 3)
    rgb = (x >> np.uint64(56)).astype(np.uint32)
    px = rgb[:, 0] | (rgb[:, 1] << 8) | (rgb[:, 2] << 16) | np.uint32(255 << 24)
    return px.astype(np.uint32).reshape(height, width)


# ---- camera ------------------------------------------------------------------------------

def view_matrix_from_colmap(quat_wxyz, translation) -> np.ndarray:
    """mtl_engine.mm:637-659: [R | t] column-major, R from (w, x, y, z). Returns 4x4 [col][row]."""
    w, x, y, z = (np.float32(v) for v in quat_wxyz)
    one, two = np.float32(1), np.float32(2)
    m = np.zeros((4, 4), dtype=np.float32)
    m[0, :3] = [one - two * (y * y + z * z), two * (x * y + w * z), two * (x * z - w * y)]
    m[1, :3] = [two * (x * y - w * z), one - two * (x * x + z * z), two * (y * z + w * x)]
    m[2, :3] = [two * (x * z + w * y), two * (y * z - w * x), one - two * (x * x + y * y)]
    m[3, :3] = np.asarray(translation, dtype=np.float32)
    m[3, 3] = one
    return m


def projection_from_colmap(fx, fy, cx, cy, width, height, near=0.1, far=1000.0) -> np.ndarray:
    """mtl_engine.mm:662-682. Returns 4x4 [col][row] float32."""
    f32 = np.float32
    fx, fy, cx, cy = f32(fx), f32(fy), f32(cx), f32(cy)
    w, h, n, f = f32(width), f32(height), f32(near), f32(far)
    m = np.zeros((4, 4), dtype=np.float32)
    m[0, 0] = f32(2) * fx / w
    m[1, 1] = f32(2) * fy / h
    m[2, 0] = f32(2) * cx / w - f32(1)
    m[2, 1] = f32(2) * cy / h - f32(1)
    m[2, 2] = f / (f - n)
    m[2, 3] = f32(1)
    m[3, 2] = -(f * n) / (f - n)
    return m


def _matmul_colmajor(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(A*B) for [col][row] float32 matrices, summed in k order."""
    out = np.zeros((4, 4), dtype=np.float32)
    for j in range(4):
        for i in range(4):
            s = np.float32(0)
            for k in range(4):
                s = np.float32(s + np.float32(a[k, i] * b[j, k]))
            out[j, i] = s
    return out


def make_uniforms(width: int, height: int, fx: float | None = None, fy: float | None = None,
                  cx: float | None = None, cy: float | None = None,
                  quat_wxyz=(1.0, 0.0, 0.0, 0.0), translation=(0.0, 0.0, 0.0)) -> np.ndarray:
    """TiledUniforms (240 B) as a 60-element float32 array (the u32 fields viewed in place)."""
    fx = float(width) if fx is None else fx
    fy = float(width) if fy is None else fy
    cx = width / 2.0 if cx is None else cx
    cy = height / 2.0 if cy is None else cy
    view = view_matrix_from_colmap(quat_wxyz, translation)
    proj = projection_from_colmap(fx, fy, cx, cy, width, height)
    vp = _matmul_colmajor(proj, view)
    u = np.zeros(U_FLOATS, dtype=np.float32)
    u[0:16] = view.reshape(-1)
    u[16:32] = proj.reshape(-1)
    u[32:48] = vp.reshape(-1)
    u[48:50] = [width, height]
    u[50:52] = [fx, fy]
    r = view[:3, :3]  # [col][row]; R^T t: (R^T)[i] = sum_k R[i][k] t_k with R[i] = column i
    t = np.asarray(translation, dtype=np.float32)
    u[52:55] = [-(np.float32(r[i, 0] * t[0]) + np.float32(r[i, 1] * t[1]) + np.float32(r[i, 2] * t[2]))
                for i in range(3)]
    tiles = u[56:60].view(np.uint32)
    tx, ty = tiles_for(width, height)
    tiles[0], tiles[1], tiles[2], tiles[3] = tx, ty, 0, 0
    return u


def rig_camera_center(j: int) -> tuple[float, float, float]:
    """Camera j of the 8-camera rig of configs 2/4: C_j = (0.25 (j - 3.5), 0, 0)."""
    return (0.25 * (j - 3.5), 0.0, 0.0)


def rig_uniforms(j: int, width: int, height: int) -> np.ndarray:
    c = rig_camera_center(j)
    return make_uniforms(width, height, translation=(-c[0], -c[1], -c[2]))


def axis_angle_quat(axis, degrees: float) -> tuple[float, float, float, float]:
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    h = math.radians(degrees) / 2.0
    return (math.cos(h), *(math.sin(h) * a))


def general_camera(width: int, height: int) -> dict:
    """A camera that exercises every term of the projection the rig does not: a 15-degree rotation
    about a skew axis (W != I in T = J W, tiled_shaders.metal:218-225, and W^T in the world-position
    gradient, :556-565), a translation, fx != fy and an off-centre principal point
    (projectionFromColmap, mtl_engine.mm:662-682). Keyword arguments of make_uniforms and
    synthetic_gaussians_camera."""
    return dict(fx=0.9635 * width, fy=0.8958 * width, cx=0.526 * width, cy=0.479 * height,
                quat_wxyz=axis_angle_quat((1.0, 2.0, 0.5), 15.0), translation=(0.3, -0.2, 0.5))


CONFIGS = {
    1: dict(n=10_000, width=256, height=256, seed=1, views=1),
    2: dict(n=100_000, width=1920, height=1080, seed=2, views=1),
    3: dict(n=1_000_000, width=1920, height=1080, seed=3, views=1),
    4: dict(n=1_000_000, width=1920, height=1080, seed=3, views=8),
    5: dict(n=5_000_000, width=1920, height=1080, seed=5, views=8),
}
