import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def coracle():
    """The C restatement (oracle/), built on demand.  Test infrastructure only."""
    so = os.path.join(ROOT, "oracle", "libsalamander_ref.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from oracle.salamander_ref import COracle
    return COracle(so)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "salamander_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(ROOT, "tests", "golden", "batch_digests.json")) as f:
        dig = json.load(f)
    return vec, dig


@pytest.fixture(scope="session")
def gpu():
    """cuda:0 plus a loaded libhyobfs; fails (not skips) when the GPU tier runs without them."""
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs a GPU"
    import hysteria_amd
    assert hysteria_amd.device_count() > 0
    return torch.device("cuda:0")
