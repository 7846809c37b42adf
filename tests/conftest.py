import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "self-supervise-sfm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: full-size CPU oracle runs (tens of seconds)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
