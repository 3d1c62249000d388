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
