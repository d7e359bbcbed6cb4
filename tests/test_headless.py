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
