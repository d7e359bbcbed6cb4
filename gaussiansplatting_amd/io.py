"""Scene formats and initialisation over the C-ABI (host-side C++ in the
library: gaussiansplatting_amd/csrc/gs_io.cpp), plus a COLMAP binary writer for synthetic scenes.

  load_colmap             loadColmap (colmap_loader.cpp:185-191)
  scene_extent            computeSceneExtent (:232-264)
  gaussians_from_colmap   gaussiansFromColmap (main.mm:59-187)
  colmap_uniforms         the TiledUniforms of one COLMAP view (mtl_engine.mm:637-682, 866-924)
  load_ply / save_ply     load_ply (ply_loader.cpp:61-290) / PLYExporter (ply_exporter.hpp:18-163)
  save_ppm                saveTextureToPPM (mtl_engine.mm:19-63)
  write_colmap            COLMAP's binary model format (cameras.bin, images.bin, points3D.bin)
"""
from __future__ import annotations

import ctypes
import os
import struct
from ctypes import byref, c_float, c_uint32, c_uint64, c_void_p

import numpy as np

from . import _lib
from .scene import G_FLOATS, U_FLOATS


class ColmapScene:
    """A loaded COLMAP model (handle owned by the library)."""

    def __init__(self, path: str):
        self._h = c_void_p()
        _lib.call("gs_colmap_load", os.fsencode(path), byref(self._h))
        nc, ni, npt = c_uint32(), c_uint32(), c_uint64()
        _lib.call("gs_colmap_counts", self._h, byref(nc), byref(ni), byref(npt))
        self.cameras = {}
        for i in range(nc.value):
            cam = _lib.GsColmapCamera()
            _lib.call("gs_colmap_camera", self._h, i, byref(cam))
            self.cameras[cam.id] = cam
        self.images = []
        for i in range(ni.value):
            im = _lib.GsColmapImage()
            _lib.call("gs_colmap_image", self._h, i, byref(im))
            self.images.append(im)
        pts = (_lib.GsColmapPoint * max(npt.value, 1))()
        _lib.call("gs_colmap_points", self._h, ctypes.cast(pts, c_void_p), npt.value)
        arr = np.ctypeslib.as_array(ctypes.cast(pts, ctypes.POINTER(c_float)), shape=(max(npt.value, 1), 7))
        self.points = arr[:npt.value].copy()  # (n, 7): position xyz, colour rgb, error

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().gs_colmap_free(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def scene_extent(self) -> float:
        e = c_float()
        _lib.call("gs_colmap_scene_extent", self._h, byref(e))
        return float(e.value)

    def camera_position(self, index: int) -> np.ndarray:
        out = (c_float * 3)()
        _lib.call("gs_colmap_camera_position", byref(self.images[index]), out)
        return np.array(out[:], dtype=np.float32)

    def gaussians(self, scene_extent: float | None = None) -> np.ndarray:
        """gaussiansFromColmap: (N, 28) float32 Gaussian records."""
        ext = self.scene_extent() if scene_extent is None else scene_extent
        n = c_uint64()
        _lib.call("gs_gaussians_from_colmap", self._h, float(ext), None, 0, byref(n))
        g = np.zeros((max(n.value, 1), G_FLOATS), dtype=np.float32)
        _lib.call("gs_gaussians_from_colmap", self._h, float(ext), g.ctypes.data, n.value, byref(n))
        return g[:n.value]

    def uniforms(self, index: int, width: int | None = None, height: int | None = None) -> np.ndarray:
        im = self.images[index]
        cam = self.cameras[im.camera_id]
        w = cam.width if width is None else width
        h = cam.height if height is None else height
        u = np.zeros(U_FLOATS, dtype=np.float32)
        _lib.call("gs_colmap_uniforms", byref(cam), byref(im), int(w), int(h), u.ctypes.data)
        return u


def load_colmap(path: str) -> ColmapScene:
    return ColmapScene(path)


def load_ply(path: str) -> np.ndarray:
    n = c_uint64()
    _lib.call("gs_ply_load", os.fsencode(path), None, 0, byref(n))
    g = np.zeros((max(n.value, 1), G_FLOATS), dtype=np.float32)
    _lib.call("gs_ply_load", os.fsencode(path), g.ctypes.data, n.value, byref(n))
    return g[:n.value]


def save_ply(path: str, gaussians: np.ndarray) -> int:
    g = np.ascontiguousarray(gaussians, dtype=np.float32)
    nw = c_uint64()
    _lib.call("gs_ply_save", os.fsencode(path), g.ctypes.data, g.shape[0], byref(nw))
    return int(nw.value)


def save_ppm(path: str, rgba8: np.ndarray) -> None:
    img = np.ascontiguousarray(rgba8).view(np.uint32)
    h, w = img.shape
    _lib.call("gs_ppm_save", os.fsencode(path), img.ctypes.data, w, h)


def load_ppm(path: str) -> np.ndarray:
    """A P6 PPM as an (H, W) uint32 RGBA8 image (alpha 255), gs_ppm_load."""
    from ctypes import c_uint32
    w, h = c_uint32(), c_uint32()
    _lib.call("gs_ppm_load", os.fsencode(path), None, 0, byref(w), byref(h))
    img = np.zeros((h.value, w.value), dtype=np.uint32)
    _lib.call("gs_ppm_load", os.fsencode(path), img.ctypes.data, img.size, byref(w), byref(h))
    return img


def write_colmap(path: str, cameras, images, points) -> None:
    """COLMAP binary model writer (the layout colmap_loader.cpp reads).

    cameras: list of (id, model, width, height, params); images: list of
    (id, (qw, qx, qy, qz), (tx, ty, tz), camera_id, name); points: (N, 6) array of xyz + rgb8
    (ids 1..N, error 0, empty tracks)."""
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "cameras.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(cameras)))
        for cid, model, w, h, params in cameras:
            f.write(struct.pack("<IiQQ", cid, model, w, h))
            f.write(struct.pack(f"<{len(params)}d", *params))
    with open(os.path.join(path, "images.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(images)))
        for iid, q, t, cid, name in images:
            f.write(struct.pack("<I4d3dI", iid, *q, *t, cid))
            f.write(name.encode() + b"\0")
            f.write(struct.pack("<Q", 0))
    pts = np.asarray(points)
    with open(os.path.join(path, "points3D.bin"), "wb") as f:
        f.write(struct.pack("<Q", pts.shape[0]))
        rec = np.zeros(pts.shape[0], dtype=np.dtype([("id", "<u8"), ("xyz", "<f8", 3), ("rgb", "u1", 3),
                                                      ("err", "<f8"), ("track", "<u8")]))
        rec["id"] = np.arange(1, pts.shape[0] + 1)
        rec["xyz"] = pts[:, :3]
        rec["rgb"] = np.clip(pts[:, 3:6], 0, 255).astype(np.uint8)
        f.write(rec.tobytes())


def synthetic_colmap(path: str, n: int, seed: int, width: int = 1920, height: int = 1080,
                     views: int = 8) -> None:
    """Config 2's synthetic COLMAP scene: one PINHOLE camera (fx = fy = width,
    centred principal point), `views` images at C_j = (0.25 (j - 3.5), 0, 0) with identity
    rotation (t = -C), and the seeded generator's positions as sparse points with random RGB8."""
    from .scene import synthetic_gaussians
    g = synthetic_gaussians(n, seed, width, height)
    rgb = np.random.default_rng(seed + 7).integers(0, 256, (n, 3))
    pts = np.concatenate([g[:, 0:3].astype(np.float64), rgb.astype(np.float64)], axis=1)
    cams = [(1, 1, width, height, (float(width), float(width), width / 2.0, height / 2.0))]
    imgs = []
    for j in range(views):
        c = 0.25 * (j - 3.5)
        imgs.append((j + 1, (1.0, 0.0, 0.0, 0.0), (-c, 0.0, 0.0), 1, f"view_{j:03d}.png"))
    write_colmap(path, cams, imgs, pts)


def synthetic_colmap_posed(path: str, n: int, seed: int, width: int = 1920, height: int = 1080,
                           views: int = 8) -> list:
    """A COLMAP scene whose images carry rotated poses and whose PINHOLE camera has fx != fy and an
    off-centre principal point (what real reconstructions give viewMatrixFromColmap /
    projectionFromColmap, mtl_engine.mm:637-682). The points are the seeded generator's draws for
    image 0's camera (scene.general_camera); image j is rotated by 15 + 2.5 j degrees about a skew
    axis and placed on a short arc, so every view sees most of the points. Returns the images'
    (quaternion, translation) poses."""
    from .scene import axis_angle_quat, general_camera, synthetic_gaussians_camera
    cam = general_camera(width, height)
    g = synthetic_gaussians_camera(n, seed, width, height, **cam)
    rgb = np.random.default_rng(seed + 7).integers(0, 256, (n, 3))
    pts = np.concatenate([g[:, 0:3].astype(np.float64), rgb.astype(np.float64)], axis=1)
    cams = [(1, 1, width, height, (cam["fx"], cam["fy"], cam["cx"], cam["cy"]))]
    imgs, poses = [], []
    for j in range(views):
        q = cam["quat_wxyz"] if j == 0 else axis_angle_quat((1.0, 2.0, 0.5), 15.0 + 2.5 * j)
        t = tuple(np.asarray(cam["translation"]) + np.array([0.12 * j, -0.03 * j, 0.05 * j]))
        poses.append((q, t))
        imgs.append((j + 1, q, t, 1, f"view_{j:03d}.png"))
    write_colmap(path, cams, imgs, pts)
    return poses
