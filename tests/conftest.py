import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()  # builds oracle/libsworacle.so on first use
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        with open(os.path.join(d, name)) as f:
            return json.load(f)
    return load


@pytest.fixture(scope="session")
def engine():
    """The HIP engine; GPU tests only.  Fails (never skips) when the library is missing."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test collected on a machine without a GPU")
    import concurrentproject_amd as sw
    sw.lib()
    sw.set_option("timeout", 5)   # a broken strip hand-off fails in seconds, not minutes
    return sw
