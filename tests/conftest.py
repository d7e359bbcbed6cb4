import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full-size parity (minutes)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Every gradient-bar audit of the run (tests/_helpers.py compare_gradients), one line each, so
    the per-class counts reach the log even under `pytest -q` (the driver's GPU-test record)."""
    try:
        from tests import _helpers
    except Exception:
        return
    if not _helpers.AUDITS:
        return
    tr = terminalreporter
    tr.write_sep("=", f"gradient-bar audits ({len(_helpers.AUDITS)})")
    tr.write_line("classes: plain = within 1e-4 max(|ref|, sum|terms|) of the reference's float sum; "
                  "shadow = within that bar of the fp64 shadow only (budget_shadow); group_floor / "
                  "conditioning = the widened classes (budget_widened)")
    for a in _helpers.AUDITS:
        head = f"{a['test']}" + (f" [{a['label']}]" if a["label"] else "")
        keys = ["live_entries", "plain", "shadow", "budget_shadow", "group_floor", "conditioning",
                "two_noise", "widened_budgeted", "budget_widened", "widened_gaussians", "max_ratio_to_bar"]
        body = ", ".join(f"{k} {a[k]:.4g}" if isinstance(a[k], float) else f"{k} {a[k]}"
                         for k in keys if k in a)
        tr.write_line(f"{head}: {body}")
        if a.get("widened_per_field"):
            tr.write_line(f"    widened per field: {a['widened_per_field']}")
        if a.get("shadow_per_field"):
            tr.write_line(f"    shadow per field: {a['shadow_per_field']}")
