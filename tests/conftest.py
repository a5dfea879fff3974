import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "webgpu-msm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through libmsm's HIP kernels")
    config.addinivalue_line("markers", "slow: long-running (large N)")


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "reference_kats.json")) as f:
        kats = json.load(f)
    with open(os.path.join(d, "msm_vectors.json")) as f:
        vec = json.load(f)
    return {"kats": kats, "msm": vec}
