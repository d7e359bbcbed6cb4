"""The headless C++ caller (gs_train_headless: the reference's trainStep / train sequence through the
C++ mirror classes of include/gs_tiled_rasterizer.hpp) runs end to end on the GPU, with the
reference's densification and opacity-reset conditions (mtl_engine.mm:1108-1192)."""
from __future__ import annotations

import json
import math
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "gaussiansplatting_amd", "lib", "gs_train_headless")


def _run(*args):
    out = subprocess.run([EXE, "--n", "20000", "--width", "320", "--height", "180", *args],
                         check=True, capture_output=True, text=True, timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])


@pytest.mark.gpu
def test_headless_rasterizer_only(dev):
    d = _run("--steps", "6", "--warmup", "1", "--train", "0", "--densify-every", "2")
    assert d["pairs"] > 0 and d["ms_per_step"] > 0
    assert d["applies"] == 0 and d["n"] == d["n_initial"]


@pytest.mark.gpu
@pytest.mark.parametrize("ref_moments", ["0", "1"])
def test_headless_train_densify_and_reset(dev, ref_moments):
    """Iterations 599..605 (--start-iter 598): densification at 600, 602, 604 (500 < it < 15000,
    it % 2 == 0), opacity resets at 600 and 603; clones / splits happen and the population follows
    the apply statistics exactly. --ref-moments 1: the reference's post-densify optimizer state
    (resize + zero the new tail, mtl_engine.mm:1159-1166) instead of moments that follow."""
    d = _run("--steps", "6", "--warmup", "1", "--train", "1", "--densify-every", "2",
             "--opacity-reset-every", "3", "--start-iter", "598", "--ref-moments", ref_moments)
    assert d["moments"] == ("reference" if ref_moments == "1" else "follow")
    assert d["last_iter"] == 605
    assert d["applies"] == 3 and d["opacity_resets"] == 2
    assert d["cloned"] + d["split"] > 0
    assert d["n"] == d["n_initial"] - d["pruned"] + d["cloned"] + d["split"]
    assert math.isfinite(d["loss"]) and 0.0 < d["loss"] < 1.0


@pytest.mark.gpu
def test_headless_no_densify_before_iteration_500(dev):
    d = _run("--steps", "4", "--warmup", "1", "--train", "1", "--densify-every", "2")
    assert d["applies"] == 0 and d["n"] == d["n_initial"]


def _colmap_scene(tmp_path, n=3000, seed=2, w=320, h=180, views=4):
    from gaussiansplatting_amd import io
    d = tmp_path / "colmap"
    d.mkdir()
    io.synthetic_colmap(str(d), n, seed, w, h, views=views)
    return str(d)


def _run_colmap(d, out, *args):
    r = subprocess.run([EXE, "--colmap", d, "--export-views", str(out), "--ply", str(out / "scene.ply"),
                        "--dump-gaussians", str(out / "g.bin"), *args],
                       check=True, capture_output=True, text=True, timeout=300)
    return json.loads(r.stdout.strip().splitlines()[-1])


def _ppm_rgb(path):
    from gaussiansplatting_amd import io
    return io.load_ppm(str(path)) & 0x00FFFFFF


@pytest.mark.gpu
@pytest.mark.parametrize("steps", ["0", "5"])
def test_headless_colmap_train_export_ply(dev, tmp_path, steps):
    """The reference's main() sequence from the C++ caller (main.mm:392-413): loadColmap +
    gaussiansFromColmap -> train over the images in order -> exportTrainingViews (one
    image_%04u_render.ppm per image, mtl_engine.mm:1224-1306) -> exportPLY. Every exported view is
    bit-equal to the oracle's render (RGBA8) of the final Gaussians under that image's camera, the
    initial Gaussians are gaussiansFromColmap's, and the PLY round-trips through gs_ply_load."""
    import numpy as np

    from gaussiansplatting_amd import io
    from tests._helpers import oracle_threads
    from oracle import oracle
    d = _colmap_scene(tmp_path)
    out = tmp_path / "renders"
    out.mkdir()
    r = _run_colmap(d, out, "--steps", steps, "--warmup", "0", "--train", "1")
    sc = io.load_colmap(d)
    g0 = sc.gaussians()
    assert r["scene"] == "colmap" and r["views"] == 4 and r["n_initial"] == g0.shape[0]
    assert abs(r["extent"] - sc.scene_extent()) <= 1e-6 * sc.scene_extent()
    assert r["exported_views"] == 4 and r["last_iter"] == int(steps)
    g = np.fromfile(out / "g.bin", dtype=np.float32).reshape(-1, 28)
    assert g.shape[0] == r["n"]
    if steps == "0":
        assert np.array_equal(g.view(np.uint32), g0.view(np.uint32))
    else:
        assert not np.array_equal(g, g0) and 0.0 < r["loss"] < 1.0
    for v in range(4):
        u = sc.uniforms(v, 320, 180)
        ref = oracle.forward(g, u, 320, 180, threads=oracle_threads())
        img = _ppm_rgb(out / f"image_{v + 1:04d}_render.ppm")
        assert np.array_equal(img, ref.rgba8 & 0x00FFFFFF), f"view {v}"
    sc.close()
    # PLYExporter::exportPLY -> load_ply: positions, opacity and SH bit-exact; log-scales and the
    # (normalised on load) rotation as written
    p = io.load_ply(str(out / "scene.ply"))
    assert r["ply_written"] == g.shape[0] == p.shape[0]
    for sl in (slice(0, 3), slice(12, 13), slice(13, 25)):
        assert np.array_equal(p[:, sl].view(np.uint32), g[:, sl].view(np.uint32))
    assert np.allclose(p[:, 4:7], g[:, 4:7], rtol=0, atol=0)
    q = g[:, 8:12] / np.linalg.norm(g[:, 8:12], axis=1, keepdims=True)
    assert np.allclose(p[:, 8:12], q, rtol=0, atol=2e-7)


@pytest.mark.gpu
def test_headless_colmap_ppm_ground_truth(dev, tmp_path):
    """--gt-dir: each image's ground truth from a PPM named after the image; PPMs holding the seeded
    ground truth give the identical training run (loss and final Gaussians bit-equal)."""
    import numpy as np

    from gaussiansplatting_amd import io, scene
    d = _colmap_scene(tmp_path)
    gtd = tmp_path / "gt"
    gtd.mkdir()
    for v in range(4):
        io.save_ppm(str(gtd / f"view_{v:03d}.ppm"), scene.synthetic_ground_truth(3, v, 320, 180))
    runs = []
    for extra in ([], ["--gt-dir", str(gtd)]):
        out = tmp_path / f"o{len(runs)}"
        out.mkdir()
        r = _run_colmap(d, out, "--steps", "6", "--warmup", "0", "--train", "1", "--seed", "3", *extra)
        runs.append((r, np.fromfile(out / "g.bin", dtype=np.float32)))
    assert runs[0][0]["loss"] == runs[1][0]["loss"]
    assert np.array_equal(runs[0][1].view(np.uint32), runs[1][1].view(np.uint32))
