"""The gradient-bar audit itself (tests/_helpers.py compare_gradients): its classes, budgets and the
registry tests/conftest.py prints in the terminal summary. CPU only."""
from __future__ import annotations

import numpy as np
import pytest

from gaussiansplatting_amd import scene
from tests import _helpers


def _arrays(n=2000, seed=0):
    rng = np.random.default_rng(seed)
    ref = rng.standard_normal((n, 28))
    dead = [k for k in range(28) if k not in [o for _, o in scene.GRAD_FIELDS]]
    ref[:, dead] = 0.0
    return ref, np.abs(ref) * 2.0


def test_plain_entries_registered():
    ref, ab = _arrays()
    gpu = (ref * (1.0 + 1e-6)).astype(np.float32)
    gpu[:, [k for k in range(28) if k not in [o for _, o in scene.GRAD_FIELDS]]] = 0.0
    before = len(_helpers.AUDITS)
    a = _helpers.compare_gradients(gpu, ref, ab, None, shadow_ref=ref, cond_ref=np.zeros_like(ref), label="unit")
    assert len(_helpers.AUDITS) == before + 1
    rec = _helpers.AUDITS[-1]
    assert rec["label"] == "unit" and rec["test"].endswith("test_plain_entries_registered")
    assert a["plain"] == a["live_entries"] and a["shadow"] == 0 and a["widened_budgeted"] == 0
    assert rec["budget_shadow"] >= _helpers.WIDENED_FLOOR


def test_shadow_class_counted_and_budgeted():
    ref, ab = _arrays()
    live = [o for _, o in scene.GRAD_FIELDS]
    shadow = ref.copy()
    gpu = ref.copy()
    # 20 entries where the reference's float sum is off by 1e-3 relative but the GPU sits on the
    # exact value: shadow class
    rows = np.arange(20)
    gpu[rows, 0] = ref[rows, 0]
    ref2 = ref.copy()
    ref2[rows, 0] = ref[rows, 0] * (1.0 + 1e-2)
    a = _helpers.compare_gradients(gpu.astype(np.float32), ref2, ab, None, shadow_ref=shadow,
                                   cond_ref=np.zeros_like(ref), label="shadow")
    assert a["shadow"] == 20 and a["shadow_per_field"] == {"position_x": 20}
    # beyond the shadow budget: fails
    rows = np.arange(ref.shape[0])
    ref3 = ref.copy()
    ref3[:, live] *= 1.0 + 1e-2
    with pytest.raises(AssertionError, match="fp64 shadow"):
        _helpers.compare_gradients(gpu.astype(np.float32), ref3, ab, None, shadow_ref=shadow,
                                   cond_ref=np.zeros_like(ref), label="shadow overflow")
    # the same entries with the reference's sampled noise above the bar: explained, not budgeted
    noise = np.zeros_like(ref)
    noise[:, live] = 1.0
    a = _helpers.compare_gradients(gpu.astype(np.float32), ref3, ab, noise, shadow_ref=shadow,
                                   cond_ref=np.zeros_like(ref), label="shadow explained")
    assert a["shadow"] == a["shadow_ref_noise"] == a["live_entries"] and a["shadow_unexplained"] == 0


def test_out_of_tolerance_fails():
    ref, ab = _arrays()
    gpu = ref.copy()
    gpu[3, 1] += 1.0
    with pytest.raises(AssertionError, match="out of tolerance"):
        _helpers.compare_gradients(gpu.astype(np.float32), ref, ab, None, shadow_ref=ref,
                                   cond_ref=np.zeros_like(ref), label="bad")
