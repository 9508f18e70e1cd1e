import gzip
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libsstgpu.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    opener = gzip.open if name.endswith(".gz") else open
    with opener(path, "rt") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_alphabet():
    return load_golden("alphabet.json")


@pytest.fixture(scope="session")
def golden_tables():
    return load_golden("tables.json")


@pytest.fixture(scope="session")
def golden_cases():
    return load_golden("explain_cases.json.gz")


@pytest.fixture(scope="session")
def golden_population():
    return load_golden("population.json.gz")


@pytest.fixture(scope="session")
def golden_raise_cases():
    return load_golden("raise_cases.json")
