"""The diagnostics builds compile (CPU, hipcc cross-compile for gfx950): the blend work counters
(-DGS_BLEND_STATS, scripts/blend_stats.py), the blend per-workgroup trace (-DGS_BLEND_TRACE,
scripts/blend_trace.py) and the depth-sort phase trace (-DGS_OS_TRACE, scripts/os_trace.py). They
are tooling, not product, but they read the kernels' internals and would otherwise rot unseen."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"),
         "-I" + os.path.join(ROOT, "gaussiansplatting_amd", "csrc"), "-c"]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,define", [("gs_blend.hip", "GS_BLEND_STATS"), ("gs_blend.hip", "GS_BLEND_TRACE"),
                                        ("gs_sort.hip", "GS_OS_TRACE")])
def test_diagnostics_build_compiles(tmp_path, src, define):
    out = tmp_path / (src + ".o")
    cmd = [HIPCC, *FLAGS, "-D" + define, os.path.join(ROOT, "gaussiansplatting_amd", "csrc", src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert out.exists() and out.stat().st_size > 0
    shutil.rmtree(tmp_path, ignore_errors=True)
