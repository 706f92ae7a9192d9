import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmli_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_sessionfinish(session, exitstatus):
    """MLI_MARGINS_OUT=<path>: write the parity margins the session measured (tests/margins.py)."""
    out = os.environ.get("MLI_MARGINS_OUT")
    if not out:
        return
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import json
    import margins
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"exitstatus": int(exitstatus), "records": margins.RECORDS}, f, indent=1)


def load_golden(name):
    import torch
    return torch.load(os.path.join(GOLDEN, name + ".pt"), weights_only=True)


@pytest.fixture
def golden():
    return load_golden
