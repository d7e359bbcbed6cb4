"""Scene formats and initialisation, host-side, over the C-ABI.

Each reader/writer is checked against an independent numpy restatement of the reference code it
replaces (colmap_loader.cpp, main.mm:18-187, mtl_engine.mm:637-682 / 866-924, ply_loader.cpp,
ply_exporter.hpp, mtl_engine.mm:19-63) on synthetic files written here."""
from __future__ import annotations

import os
import struct

import numpy as np
import pytest

from gaussiansplatting_amd import io, scene

f32 = np.float32


def _cam_pos(q, t):
    qw, qx, qy, qz = (f32(v) for v in q)
    tx, ty, tz = (f32(v) for v in t)
    one, two = f32(1), f32(2)
    r00 = one - two * (qy * qy + qz * qz); r01 = two * (qx * qy - qz * qw); r02 = two * (qx * qz + qy * qw)
    r10 = two * (qx * qy + qz * qw); r11 = one - two * (qx * qx + qz * qz); r12 = two * (qy * qz - qx * qw)
    r20 = two * (qx * qz - qy * qw); r21 = two * (qy * qz + qx * qw); r22 = one - two * (qx * qx + qy * qy)
    return np.array([-(r00 * tx + r10 * ty + r20 * tz), -(r01 * tx + r11 * ty + r21 * tz),
                     -(r02 * tx + r12 * ty + r22 * tz)], dtype=np.float32)


def _mean_nn3(p, i):
    d = p - p[i]
    dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]).astype(np.float32)
    dist = np.delete(dist, i)
    if dist.size == 0:
        return f32(0.1)
    k = np.sort(dist)[:3][::-1]  # popped largest first
    s = f32(0)
    for v in k:
        s = f32(s + v)
    return f32(s / f32(k.size))


@pytest.fixture()
def colmap_dir(tmp_path):
    rng = np.random.default_rng(4)
    pts = np.concatenate([rng.normal(0, 2, (300, 3)), rng.integers(0, 256, (300, 3))], axis=1)
    cams = [(3, 1, 1600, 900, (1500.0, 1490.0, 800.0, 450.0)),
            (1, 0, 800, 600, (700.0, 400.0, 300.0)),
            (2, 2, 640, 480, (600.0, 320.0, 240.0, 0.01))]
    qs = rng.normal(0, 1, (5, 4))
    qs /= np.linalg.norm(qs, axis=1, keepdims=True)
    imgs = [(i + 10, tuple(qs[i]), tuple(rng.normal(0, 3, 3)), [3, 1, 2, 1, 3][i], f"img_{i}.jpg")
            for i in range(5)]
    io.write_colmap(str(tmp_path), cams, imgs, pts)
    return str(tmp_path), cams, imgs, pts


def test_colmap_load(colmap_dir):
    path, cams, imgs, pts = colmap_dir
    s = io.load_colmap(path)
    assert sorted(s.cameras) == [1, 2, 3]
    c3, c1, c2 = s.cameras[3], s.cameras[1], s.cameras[2]
    assert (c3.width, c3.height, c3.fx, c3.fy, c3.cx, c3.cy) == (1600, 900, f32(1500), f32(1490), f32(800), f32(450))
    assert (c1.fx, c1.fy, c1.cx, c1.cy) == (f32(700), f32(700), f32(400), f32(300))  # SIMPLE_PINHOLE
    assert (c2.fx, c2.cx) == (f32(600), f32(320))                                      # SIMPLE_RADIAL
    assert [im.id for im in s.images] == [10, 11, 12, 13, 14]
    assert s.images[2].name.decode() == "img_2.jpg" and s.images[2].camera_id == 2
    for im, (_, q, t, _, _) in zip(s.images, imgs):
        assert np.array_equal(np.array(im.rotation[:]), np.array(q, np.float32))
        assert np.array_equal(np.array(im.translation[:]), np.array(t, np.float32))
    assert s.points.shape == (300, 7)
    assert np.array_equal(s.points[:, :3], pts[:, :3].astype(np.float32))
    assert np.array_equal(s.points[:, 3:6], (pts[:, 3:6].astype(np.uint8) / f32(255)).astype(np.float32))
    # camera centres and scene extent (colmap_loader.cpp:200-264)
    cps = np.stack([_cam_pos(q, t) for _, q, t, _, _ in imgs])
    for i in range(5):
        assert np.array_equal(s.camera_position(i), cps[i])
    cen = np.zeros(3, np.float32)
    for p in cps:
        cen = (cen + p).astype(np.float32)
    cen = (cen / f32(5)).astype(np.float32)
    md = f32(0)
    for p in cps:
        d = (p - cen).astype(np.float32)
        md = max(md, f32(np.sqrt(f32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))
    assert s.scene_extent() == f32(md * f32(1.1))


def test_gaussians_from_colmap_all_points(colmap_dir):
    path, _, _, pts = colmap_dir
    s = io.load_colmap(path)
    ext = s.scene_extent()
    g = s.gaussians(ext)
    p = pts[:, :3].astype(np.float32)
    for i in range(0, 300, 7):
        sc = min(max(_mean_nn3(p, i), f32(0.0001) * f32(ext)), f32(0.1) * f32(ext))
        ls = np.float32(np.log(np.float64(sc)))  # logf is correctly rounded in glibc
        assert abs(int(g[i, 4].view(np.int32)) - int(ls.view(np.int32))) <= 1
        assert g[i, 4] == g[i, 5] == g[i, 6]
    assert np.array_equal(g[:, 0:3], p)
    assert np.all(g[:, 8] == 1) and not g[:, 9:12].any() and not g[:, 12].any()
    col = s.points[:, 3:6]
    c0 = f32(0.28209479177387814)
    assert np.array_equal(g[:, 13], ((col[:, 0] - f32(0.5)) / c0).astype(np.float32))
    assert np.array_equal(g[:, 21], ((col[:, 2] - f32(0.5)) / c0).astype(np.float32))
    assert not g[:, [14, 15, 16, 18, 19, 20, 22, 23, 24]].any()


def test_gaussians_from_colmap_sampled_median(tmp_path):
    n = 10050  # > 10000: median of a strided sample (main.mm:90-111)
    io.synthetic_colmap(str(tmp_path), n, 6, 320, 200, views=3)
    s = io.load_colmap(str(tmp_path))
    ext = s.scene_extent()
    g = s.gaussians(ext)
    p = s.points[:, :3]
    step = n // 1000
    samples = np.sort(np.array([_mean_nn3(p, i) for i in range(0, n, step)], np.float32))
    med = samples[samples.size // 2]
    sc = min(max(med, f32(0.0001) * f32(ext)), f32(0.1) * f32(ext))
    assert np.all(g[:, 4] == g[0, 4])
    assert abs(int(g[0, 4].view(np.int32)) - int(np.float32(np.log(np.float64(sc))).view(np.int32))) <= 1


def test_colmap_uniforms_match_scene_restatement(colmap_dir):
    path, _, imgs, _ = colmap_dir
    s = io.load_colmap(path)
    for i in (0, 2):
        im = s.images[i]
        cam = s.cameras[im.camera_id]
        w, h = 960, 540
        u = s.uniforms(i, w, h)
        sx, sy = f32(w) / f32(cam.width), f32(h) / f32(cam.height)
        want = scene.make_uniforms(w, h, fx=f32(cam.fx) * sx, fy=f32(cam.fy) * sy, cx=f32(cam.cx) * sx,
                                   cy=f32(cam.cy) * sy, quat_wxyz=tuple(im.rotation[:]),
                                   translation=tuple(im.translation[:]))
        assert np.array_equal(u.view(np.uint32), want.view(np.uint32))


def test_posed_colmap_scene(tmp_path):
    """io.synthetic_colmap_posed: image 0's uniforms equal scene.general_camera's bit for bit, the
    other images' rotations are not the identity, and every view sees most points (oracle)."""
    from oracle import oracle as o
    w, h = 240, 136
    poses = io.synthetic_colmap_posed(str(tmp_path), 3000, 4, w, h)
    s = io.load_colmap(str(tmp_path))
    want = scene.make_uniforms(w, h, **scene.general_camera(w, h))
    assert np.array_equal(s.uniforms(0, w, h).view(np.uint32), want.view(np.uint32))
    g = s.gaussians()
    for v in (0, 4, 7):
        u = s.uniforms(v, w, h)
        rot = u[0:16].reshape(4, 4)[:3, :3]
        assert np.abs(rot - np.eye(3)).max() > 0.2  # a real rotation
        assert abs(float(u[50]) - float(u[51])) > 5.0  # fx != fy
        pr = o.project(g, u, w, h).view(scene.PROJECTED_DTYPE).reshape(-1)
        assert (pr["radius"] > 0).mean() > 0.5, v
    assert len(poses) == 8


def _ply_bytes_reference(g):
    """ply_exporter.hpp:18-163, restated."""
    ok = ~np.isnan(g[:, 0]) & ~np.isinf(g[:, 0]) & (np.abs(g[:, 0]) < 1e6)
    v = g[ok]
    hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {v.shape[0]}"]
    hdr += [f"property float {p}" for p in ("x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2")]
    hdr += [f"property float f_rest_{i}" for i in range(9)]
    hdr += [f"property float {p}" for p in ("opacity", "scale_0", "scale_1", "scale_2",
                                            "rot_0", "rot_1", "rot_2", "rot_3")]
    hdr += ["end_header"]
    z = np.zeros((v.shape[0], 3), np.float32)
    sh = v[:, 13:25]
    rest = sh[:, [1, 5, 9, 2, 6, 10, 3, 7, 11]]
    rows = np.concatenate([v[:, 0:3], z, sh[:, [0, 4, 8]], rest, v[:, 12:13], v[:, 4:7], v[:, 8:12]], axis=1)
    return ("\n".join(hdr) + "\n").encode() + rows.astype("<f4").tobytes()


def test_ply_save_and_load(tmp_path):
    g = scene.synthetic_gaussians(500, 9, 64, 64)
    g[:, 14:17] = np.random.default_rng(1).normal(0, 1, (500, 3))
    g[7, 0] = np.nan
    g[8, 0] = 2e6
    path = str(tmp_path / "g.ply")
    assert io.save_ply(path, g) == 498
    assert open(path, "rb").read() == _ply_bytes_reference(g)
    back = io.load_ply(path)
    keep = np.ones(500, bool)
    keep[[7, 8]] = False
    want = g[keep].copy()
    # load_ply normalises quaternions (ply_loader.cpp:208-214); the generator's are unit already
    q = want[:, 8:12]
    ln = np.sqrt(q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1] + q[:, 2] * q[:, 2] + q[:, 3] * q[:, 3]).astype(np.float32)
    want[:, 8:12] = (q / ln[:, None]).astype(np.float32)
    want[:, 4:7] = np.clip(want[:, 4:7], -8, 8)
    want[:, 3] = want[:, 7] = 0
    want[:, 25:] = 0
    assert np.array_equal(back, want)


def test_ply_ascii_linear_scales_and_dc_only(tmp_path):
    # ascii, linear scales (all in (0, 1]) -> log, no f_rest -> higher SH zero, a zero quaternion
    props = ["x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "opacity", "scale_0", "scale_1", "scale_2",
             "rot_0", "rot_1", "rot_2", "rot_3"]
    rows = [[1, 2, 3, 0.1, 0.2, 0.3, -1.0, 0.5, 0.25, 1.0, 0, 0, 0, 0],
            [4, 5, 6, -0.1, 0.0, 0.3, 2.0, 0.01, 0.02, 0.03, 2, 0, 0, 0]]
    txt = "ply\nformat ascii 1.0\ncomment test\nelement vertex 2\n"
    txt += "".join(f"property float {p}\n" for p in props) + "end_header\n"
    txt += "".join(" ".join(str(v) for v in r) + "\n" for r in rows)
    path = tmp_path / "a.ply"
    path.write_text(txt)
    g = io.load_ply(str(path))
    assert g.shape == (2, 28)
    assert np.array_equal(g[0, 4:7], np.array([np.log(f32(0.5)), np.log(f32(0.25)), np.log(f32(1.0))], np.float32))
    assert np.array_equal(g[0, 8:12], np.array([1, 0, 0, 0], np.float32))
    assert np.array_equal(g[1, 8:12], np.array([1, 0, 0, 0], np.float32))
    assert g[1, 12] == 2.0 and g[0, 13] == f32(0.1) and g[0, 17] == f32(0.2) and g[0, 21] == f32(0.3)
    assert not g[:, [14, 15, 16, 18, 19, 20, 22, 23, 24]].any()


def test_ply_ascii_single_digits_no_final_newline(tmp_path):
    """A valid ASCII PLY whose values are single characters and whose last row has no trailing
    newline is loaded (the truncation bound counts one byte per value)."""
    props = ["x", "y", "z", "f_dc_0", "f_dc_1", "f_dc_2", "opacity", "scale_0", "scale_1", "scale_2",
             "rot_0", "rot_1", "rot_2", "rot_3"]
    txt = "ply\nformat ascii 1.0\nelement vertex 1\n"
    txt += "".join(f"property float {p}\n" for p in props) + "end_header\n"
    txt += " ".join(["0"] * 10 + ["1", "0", "0", "0"])  # 27 bytes for 14 values, no newline
    path = tmp_path / "tight.ply"
    path.write_text(txt)
    g = io.load_ply(str(path))
    assert g.shape == (1, 28) and g[0, 8] == 1.0 and not g[0, 0:3].any()


def test_ppm_save(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 2 ** 32, (5, 7), dtype=np.uint64).astype(np.uint32)
    path = str(tmp_path / "x.ppm")
    io.save_ppm(path, img)
    data = open(path, "rb").read()
    hdr = b"P6\n7 5\n255\n"
    assert data[:len(hdr)] == hdr
    rgb = np.frombuffer(data[len(hdr):], np.uint8).reshape(5, 7, 3)
    assert np.array_equal(rgb[..., 0], (img & 0xFF).astype(np.uint8))
    assert np.array_equal(rgb[..., 2], ((img >> 16) & 0xFF).astype(np.uint8))


def test_ppm_load_round_trip_and_malformed(tmp_path):
    from gaussiansplatting_amd._lib import GS_E_INVALID, GsError
    rng = np.random.default_rng(4)
    img = rng.integers(0, 2 ** 24, (9, 13), dtype=np.uint64).astype(np.uint32) | np.uint32(255 << 24)
    path = str(tmp_path / "a.ppm")
    io.save_ppm(path, img)
    assert np.array_equal(io.load_ppm(path), img)
    # comments and arbitrary whitespace in the header
    rgb = np.dstack([(img >> s) & 0xFF for s in (0, 8, 16)]).astype(np.uint8)
    (tmp_path / "c.ppm").write_bytes(b"P6 # c\n13\t9\n# more\n255\n" + rgb.tobytes())
    assert np.array_equal(io.load_ppm(str(tmp_path / "c.ppm")), img)
    bad = {"magic": b"P3\n1 1\n255\n\0\0\0", "maxval": b"P6\n1 1\n65535\n\0\0\0\0\0\0",
           "trunc": b"P6\n4 4\n255\n\0\0\0", "huge": b"P6\n99999999 99999999\n255\n",
           "neg": b"P6\n-1 2\n255\n", "empty": b"", "hdr": b"P6\n3"}
    for name, data in bad.items():
        p = tmp_path / f"{name}.ppm"
        p.write_bytes(data)
        with pytest.raises(GsError) as e:
            io.load_ppm(str(p))
        assert e.value.code == GS_E_INVALID, name


def test_colmap_missing_file_fails_loudly(tmp_path):
    from gaussiansplatting_amd._lib import GsError
    with pytest.raises(GsError):
        io.load_colmap(str(tmp_path / "nope"))


def test_malformed_ply_rejected(tmp_path):
    """Lying vertex counts (2^60+1 over 12 MB of rows, 2^44, 2^64-1), truncated rows, oversized
    elements before the vertices, list/unknown property types: GS_E_INVALID, no allocation of what
    the header claims, no crash (the reader trusted the header's count)."""
    from gaussiansplatting_amd._lib import GS_E_INVALID, GsError
    from tests import _malformed
    for name, path in sorted(_malformed.ply_cases(str(tmp_path)).items()):
        with pytest.raises(GsError) as e:
            io.load_ply(path)
        assert e.value.code == GS_E_INVALID, name


def test_malformed_colmap_rejected(tmp_path):
    """Lying camera / image / point / 2D-point / track counts and truncated records."""
    from gaussiansplatting_amd._lib import GS_E_INVALID, GsError
    from tests import _malformed
    s = io.load_colmap(_malformed.colmap_good(str(tmp_path)))
    assert len(s.cameras) == 1 and len(s.images) == 2 and s.points.shape == (5, 7)
    for name, path in sorted(_malformed.colmap_cases(str(tmp_path)).items()):
        with pytest.raises(GsError) as e:
            io.load_colmap(path)
        assert e.value.code == GS_E_INVALID, name
