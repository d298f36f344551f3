import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    return load


@pytest.fixture
def dbg():
    """The library's explicit debug options (bgx_debug_option, include/bgx.h) with a
    monkeypatch-like interface; every option set is unset at teardown."""
    from bgx import _lib

    class Dbg:
        def __init__(self):
            self.names = set()

        def setenv(self, name, value):
            _lib.debug_option(name, value)
            self.names.add(name)

        def delenv(self, name, raising=True):
            _lib.debug_option(name, None)

    d = Dbg()
    yield d
    for n in d.names:
        _lib.debug_option(n, None)
