import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        p = os.path.join(GOLDEN, name)
        if name.endswith(".json"):
            return json.load(open(p))
        return open(p, "rb").read()
    return load


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build(ref=os.path.isdir("/root/reference/src"))
    return oracle


@pytest.fixture(scope="session")
def engine():
    """The GPU engine, bound to device 0.  Fails (not skips) when a gpu test
    runs without the built library or device: there is no CPU fallback."""
    import librdkafka_amd as L
    if not os.path.exists(L.LIB_PATH):
        L.build()
    L.init(0)
    return L
