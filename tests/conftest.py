import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsail_hip.so on the device)")


@pytest.fixture(scope="session")
def fixtures():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "fixtures.json")) as f:
        return json.load(f)
