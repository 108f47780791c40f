import os
import sys

import pytest
# torch before the product library in every test process (as bench.py and
# INTEGRATION.md do): both link SONAME libamdhip64.so.7, and whichever loads
# first is the HIP runtime the other binds to; tests that hand torch tensors and
# streams to the library need torch's.
import torch  # noqa: F401

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "oracle", "scenes", "bidirectional-path-tracing_amd"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available() -> bool:
    try:
        import bdpt_amd
        return bdpt_amd.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_manifest():
    import json
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
        return json.load(f)


def load_golden(name):
    import numpy as np
    return np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))["fb"]
