"""Malformed scene files for the parsers of gs_io.cpp (COLMAP binary model, 3DGS PLY): lying
headers, truncated data, wrong types. Shared by tests/test_io.py (the product library must return
GS_E_INVALID, never crash or allocate what the header claims) and tests/test_sanitize.py (the same
files under AddressSanitizer + UndefinedBehaviorSanitizer).

The formats are the reference's readers' (colmap_loader.cpp:26-189, ply_loader.cpp:61-290)."""
from __future__ import annotations

import os
import struct

import numpy as np

PLY_PROPS = ["x", "y", "z", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3",
             "opacity", "f_dc_0", "f_dc_1", "f_dc_2", "nx", "ny"]  # 16 float properties


def _ply_header(count, props=PLY_PROPS, fmt="binary_little_endian", extra=""):
    h = f"ply\nformat {fmt} 1.0\n{extra}element vertex {count}\n"
    h += "".join(f"property float {p}\n" for p in props)
    return (h + "end_header\n").encode()


def _rows(n, props=PLY_PROPS):
    r = np.zeros((n, len(props)), np.float32)
    r[:, 6] = 1.0  # unit quaternion
    return r.tobytes()


def ply_cases(d: str) -> dict[str, str]:
    """name -> path of a malformed PLY file."""
    cases = {
        # the advisor's reproducers: a 2^60+1 vertex header over ~12 MB of rows, and 2^44 vertices
        "ply_count_2p60": _ply_header(2 ** 60 + 1) + _rows(200_000),
        "ply_count_2p44": _ply_header(2 ** 44) + _rows(10),
        "ply_count_wraps": _ply_header(2 ** 64 - 1) + _rows(10),
        "ply_negative_count": _ply_header(-5) + _rows(10),
        "ply_truncated_rows": _ply_header(100) + _rows(99) + b"\0" * 20,
        "ply_ascii_count_2p60": _ply_header(2 ** 60, fmt="ascii") + b"0 " * 64 + b"\n",
        "ply_ascii_truncated": _ply_header(3, fmt="ascii") + b"1 2 3\n",
        "ply_element_before_vertex_2p62": (b"ply\nformat binary_little_endian 1.0\nelement face 4611686018427387904\n"
                                           b"property float a\n" + _ply_header(2)[len(b"ply\nformat binary_little_endian 1.0\n"):]
                                           + _rows(2)),
        "ply_ascii_element_before_vertex_2p60": (b"ply\nformat ascii 1.0\nelement face 1152921504606846976\n"
                                                 b"property float a\n" + _ply_header(1, fmt="ascii")[len(b"ply\nformat ascii 1.0\n"):]
                                                 + b"0\n"),
        "ply_list_in_vertex": b"ply\nformat binary_little_endian 1.0\nelement vertex 1\nproperty list uchar int idx\nend_header\n" + b"\0" * 8,
        "ply_bad_type": b"ply\nformat binary_little_endian 1.0\nelement vertex 1\nproperty quad x\nend_header\n" + b"\0" * 8,
        "ply_no_vertex": b"ply\nformat binary_little_endian 1.0\nend_header\n",
        "ply_big_endian": _ply_header(1, fmt="binary_big_endian") + _rows(1),
        "ply_not_ply": b"solid cube\n",
        "ply_missing_properties": _ply_header(1, props=["x", "y", "z"]) + np.zeros(3, np.float32).tobytes(),
        "ply_empty": b"",
    }
    out = {}
    for name, data in cases.items():
        p = os.path.join(d, name + ".ply")
        with open(p, "wb") as f:
            f.write(data)
        out[name] = p
    return out


def _colmap_dir(d, name, cameras: bytes, images: bytes, points: bytes) -> str:
    p = os.path.join(d, name)
    os.makedirs(p, exist_ok=True)
    for fn, data in (("cameras.bin", cameras), ("images.bin", images), ("points3D.bin", points)):
        with open(os.path.join(p, fn), "wb") as f:
            f.write(data)
    return p


def _cameras(n=1):
    return struct.pack("<Q", n) + b"".join(struct.pack("<IiQQ4d", i + 1, 1, 64, 48, 64.0, 64.0, 32.0, 24.0)
                                            for i in range(n))


def _image(iid, n2d=0, name=b"a.png", points2d=b""):
    return struct.pack("<I4d3dI", iid, 1.0, 0.0, 0.0, 0.0, 0.1 * iid, 0.0, 0.0, 1) + name + b"\0" + \
        struct.pack("<Q", n2d) + points2d


def _images(n=2):
    return struct.pack("<Q", n) + b"".join(_image(i + 1) for i in range(n))


def _point(pid, track=0, track_data=b""):
    return struct.pack("<Q3d3BdQ", pid, 0.1 * pid, 0.0, 3.0, 10, 20, 30, 0.5, track) + track_data


def _points(n=5):
    return struct.pack("<Q", n) + b"".join(_point(i + 1) for i in range(n))


def colmap_good(d: str) -> str:
    return _colmap_dir(d, "colmap_good", _cameras(), _images(), _points())


def colmap_cases(d: str) -> dict[str, str]:
    """name -> directory of a malformed COLMAP model."""
    c = {
        "colmap_cameras_count_2p60": (struct.pack("<Q", 2 ** 60) + _cameras()[8:], _images(), _points()),
        "colmap_cameras_truncated": (_cameras()[:-5], _images(), _points()),
        "colmap_images_count_2p62": (_cameras(), struct.pack("<Q", 2 ** 62) + _images()[8:], _points()),
        "colmap_images_n2d_2p62": (_cameras(), struct.pack("<Q", 1) + _image(1, n2d=2 ** 62), _points()),
        "colmap_images_n2d_wraps": (_cameras(), struct.pack("<Q", 1) + _image(1, n2d=2 ** 63 + 1), _points()),
        "colmap_images_unterminated_name": (_cameras(), struct.pack("<Q", 1) + _image(1)[:-9], _points()),
        "colmap_points_count_2p61": (_cameras(), _images(), struct.pack("<Q", 2 ** 61) + _points()[8:]),
        "colmap_points_track_2p62": (_cameras(), _images(), struct.pack("<Q", 1) + _point(1, track=2 ** 62)),
        "colmap_points_track_truncated": (_cameras(), _images(),
                                          struct.pack("<Q", 1) + _point(1, track=3, track_data=b"\0" * 16)),
        "colmap_points_empty_file": (_cameras(), _images(), b""),
    }
    return {name: _colmap_dir(d, name, *files) for name, files in c.items()}
