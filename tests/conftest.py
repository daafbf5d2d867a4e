import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsdrgpu.so on the device)")


@pytest.fixture(scope="session")
def rng():
    # one generator for the session (inputs depend on the tests that ran before); SDRGPU_TEST_SEED draws
    # another set of inputs, to check that no bar holds only for the default draw
    import numpy as np
    return np.random.default_rng(int(os.environ.get("SDRGPU_TEST_SEED", "0xACE1"), 0))
