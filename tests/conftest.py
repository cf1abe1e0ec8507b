import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the built libkfec.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle, build
    build()
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "golden.json")) as f:
        meta = json.load(f)
    arrs = np.load(os.path.join(d, "golden.npz"), allow_pickle=False)
    return meta, arrs
