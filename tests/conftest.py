import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def resources():
    return os.path.join(ROOT, "tests", "golden", "resources")


def read_fixture(base):
    out = {}
    for ext in ("inst", "wtns", "gadgets"):
        with open(base + "." + ext) as f:
            out[ext] = f.read()
    return out
