import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return torch.device("cuda:0")


def pytest_sessionfinish(session, exitstatus):
    """Write the ground-plane report (kappa and observed error per golden case, golden_cases.check_plane)."""
    gc = sys.modules.get("golden_cases")
    if gc is not None and getattr(gc, "PLANE_REPORT", None):
        import json
        out = os.path.join(REPO, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        torch = sys.modules.get("torch")
        where = "gpu" if torch is not None and torch.cuda.is_available() else "cpu"  # device path / oracle
        with open(os.path.join(out, f"plane_report_{where}.json"), "w") as f:
            json.dump({"contract": "coefficients within 1e-9 |x| + 1024 eps kappa ||x||; residual norm within "
                       "1e-9 ||z|| (tests/golden_cases.py::check_plane)", "cases": gc.PLANE_REPORT}, f, indent=1,
                      sort_keys=True)
