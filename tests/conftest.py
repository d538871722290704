import json
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: full-size model on CPU (minutes)")


def load_golden(name):
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, name + ".safetensors"))


def load_meta(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="session")
def gpu_available():
    return torch.cuda.is_available()
