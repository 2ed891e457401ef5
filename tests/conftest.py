import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libadaptive_amd.so)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz")) as z:
        return {k: z[k] for k in z.files}


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def manifest():
    return golden_manifest()


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU (run with -m 'not gpu')")
    return torch.device("cuda:0")
