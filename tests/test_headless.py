"""The headless C++ caller (gs_train_headless: the reference's trainStep sequence through the C++
mirror classes of include/gs_tiled_rasterizer.hpp) runs end to end on the GPU."""
from __future__ import annotations

import json
import math
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "gaussiansplatting_amd", "lib", "gs_train_headless")


@pytest.mark.gpu
@pytest.mark.parametrize("train", [0, 1])
def test_headless_train_step(dev, train):
    out = subprocess.run([EXE, "--n", "20000", "--width", "320", "--height", "180", "--steps", "6",
                          "--warmup", "1", "--train", str(train), "--densify-every", "2",
                          "--opacity-reset-every", "3"],
                         check=True, capture_output=True, text=True, timeout=300).stdout
    d = json.loads(out.strip().splitlines()[-1])
    assert d["pairs"] > 0 and d["ms_per_step"] > 0
    if train:
        assert math.isfinite(d["loss"]) and 0.0 < d["loss"] < 1.0
