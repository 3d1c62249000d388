import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def fixture_golden():
    return load_golden("fixture.json")


@pytest.fixture(scope="session")
def stats_golden():
    return load_golden("stats.json")


@pytest.fixture(scope="session")
def synth_golden():
    return load_golden("synth.json")


@pytest.fixture(scope="session")
def experimental_golden():
    return load_golden("experimental.json")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def lib_built():
    from metacov_amd import build
    build.build(verbose=False)
    return build.LIB


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so) beside the
    /opt/rocm one libmetacov_amd links; torch only finds the GPU when its
    runtime initialises first.  GPU runs therefore touch torch's device
    before any test creates a library context."""
    expr = request.config.getoption("-m") or ""
    if "gpu" in expr and "not gpu" not in expr:
        try:
            import torch
            if torch.cuda.is_available():
                torch.zeros(1, device="cuda")
        except Exception:   # a test that needs torch reports it itself
            pass
