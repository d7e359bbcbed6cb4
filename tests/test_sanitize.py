"""AddressSanitizer + UndefinedBehaviorSanitizer build (`make sanitize`) of the host code that parses
untrusted files — gs_io.cpp's COLMAP binary-model and PLY readers (the reference's
colmap_loader.cpp:26-189, ply_loader.cpp:61-290) — and of the CPU oracle (the host
oracle runs under ASan/UBSan). Well-formed, truncated and lying-header inputs (tests/_malformed.py);
a sanitizer report or a crash fails the test, and every malformed file must be rejected with
GS_E_INVALID."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from tests import _malformed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "san", "gs_san")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:allocator_may_return_null=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")


@pytest.fixture(scope="module")
def san():
    r = subprocess.run(["make", "-C", ROOT, "sanitize"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return EXE


def _run(exe, *args) -> str:
    r = subprocess.run([exe, *args], capture_output=True, text=True, env=ENV, timeout=300)
    report = "AddressSanitizer" in r.stderr or "LeakSanitizer" in r.stderr or "runtime error" in r.stderr
    assert not report and r.returncode == 0, f"{args}: rc={r.returncode}\n{r.stderr[-4000:]}"
    return r.stdout.strip()


def _status(out: str) -> int:
    return int(out.split()[0].split("=")[1])


def test_sanitized_parsers_reject_malformed_files(san, tmp_path):
    for name, path in sorted(_malformed.ply_cases(str(tmp_path)).items()):
        out = _run(san, "ply", path)
        assert _status(out) == -1, f"{name}: {out}"
    for name, path in sorted(_malformed.colmap_cases(str(tmp_path)).items()):
        out = _run(san, "colmap", path)
        assert _status(out) == -1, f"{name}: {out}"
    bad_ppm = {"magic": b"P3\n1 1\n255\n\0\0\0", "maxval": b"P6\n1 1\n65535\n\0\0",
               "trunc": b"P6\n4 4\n255\n\0\0\0", "huge": b"P6\n99999999 99999999\n255\n",
               "comment_eof": b"P6 # no end", "long_token": b"P6\n" + b"9" * 40 + b" 1\n255\n", "empty": b""}
    for name, data in sorted(bad_ppm.items()):
        p = tmp_path / f"{name}.ppm"
        p.write_bytes(data)
        out = _run(san, "ppm", str(p))
        assert _status(out) == -1, f"{name}: {out}"


def test_sanitized_parsers_read_valid_files(san, tmp_path):
    from gaussiansplatting_amd import io, scene
    out = _run(san, "colmap", _malformed.colmap_good(str(tmp_path)))
    assert out.startswith("status=0 cameras=1 images=2 points=5 gaussians_rc=0 uniforms_rc=0"), out
    d = tmp_path / "scene"
    io.synthetic_colmap(str(d), 2000, 3, 128, 96, views=3)
    out = _run(san, "colmap", str(d))
    assert out.startswith("status=0 cameras=1 images=3 points=2000"), out
    g = scene.synthetic_gaussians(300, 4, 64, 64)
    io.save_ply(str(tmp_path / "g.ply"), g)
    assert _run(san, "ply", str(tmp_path / "g.ply")) == "status=0 count=300"
    img = np.arange(35, dtype=np.uint32).reshape(5, 7) | np.uint32(255 << 24)
    io.save_ppm(str(tmp_path / "i.ppm"), img)
    assert _run(san, "ppm", str(tmp_path / "i.ppm")) == "status=0 size=7x5"


def test_sanitized_oracle_matches_plain_build(san):
    """The oracle (forward + backward, two OpenMP threads) under the sanitizers: no report, and the
    same P as the regular build of oracle/libgs_oracle.so."""
    from gaussiansplatting_amd import scene
    from oracle import oracle
    n, w, h, seed = 1500, 96, 64, 7
    out = _run(san, "oracle", str(n), str(w), str(h), str(seed))
    g = scene.synthetic_gaussians(n, seed, w, h)
    f = oracle.forward(g, scene.make_uniforms(w, h), w, h)
    assert out.startswith(f"status=0 pairs={f.num_pairs} "), out
    assert np.isfinite(float(out.split("grad_abs_sum=")[1]))
